#!/bin/bash
# round 5, final library (the PMC passes of profiles/pmc_*.json ran it): smoke(), every bench line
# (the default line with its CPU baseline, every workload, the one-engine variants, the match-2
# probe), then kernel traces of the main workloads.  Output: gpurun_out/r05final/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/${FINAL_TAG:-r05final}; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.json" 2> "$O/$name.err"
  local rc=$?
  echo "[$name] rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json | head -1)"
  if fatal $rc; then echo "fatal in $name"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
step bench_sw_local_start 600 python bench.py --workload sw_local_start --cpu-seconds 8
step bench_sw_local_start_s1 600 python bench.py --workload sw_local_start --streams 1 --no-cpu
step bench_sw_local_tb 600 python bench.py --workload sw_local_tb --no-cpu
step bench_sw_local_300 600 python bench.py --workload sw_local_300 --no-cpu
step bench_sw_local_match2 600 python bench.py --workload sw_local --scores 2,4,6,1 --no-cpu
step bench_nw_tb 600 python bench.py --workload nw_tb --no-cpu
step bench_nw_tb_s1 600 python bench.py --workload nw_tb --streams 1 --no-cpu
step bench_nw_score 600 python bench.py --workload nw_score --no-cpu
step bench_semi 600 python bench.py --workload semi --no-cpu
step bench_semi_start 600 python bench.py --workload semi_start --no-cpu
step bench_semi_banded 600 python bench.py --workload semi_banded --no-cpu
step bench_pairhmm 600 python bench.py --workload pairhmm --cpu-seconds 8
step bench_nvbio_gotoh 600 python bench.py --workload nvbio_gotoh --no-cpu
step bench_nvbio_banded 600 python bench.py --workload nvbio_banded --no-cpu
step bench_ksw 600 python bench.py --workload ksw --no-cpu
cd /tmp && export TMPDIR=/tmp
for w in sw_local pairhmm semi semi_start sw_local_start nw_tb; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
    python3 $ROOT/bench.py --workload $w --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_$w.json 2> $O/prof_$w.err
  rc=$?; echo "[prof $w] rc=$rc"; if fatal $rc; then exit $rc; fi
done
exit 0
