#!/bin/bash
# The final measurement session of a library, in one gpurun call: the GPU suite, the PMC passes of
# every bench workload (scripts/pmc_session.sh: separate rocprofv3 --pmc runs, never combined with
# traces) summarised on the box into profiles/pmc_<w>.json (tools/pmc_summary.py, so the bench lines
# after them carry the traffic and issue-priced figures of this same library), smoke(), every bench
# line (CPU baselines on the configs BASELINE.md quotes them for, the one-engine variants, the
# drop-in boundary line), then kernel-trace summaries.  Output: gpurun_out/$FINAL_TAG (default
# final)/, PMC copies in gpurun_out/final_pmc/.  PARTS (default "tests pmc bench prof") picks the
# parts, so the session fits gpurun's 20-minute limit in two or three calls:
#   gpurun --timeout 1200 -- 'PARTS="tests pmc" bash scripts/repro_final.sh'
#   gpurun --timeout 1200 -- 'PARTS="bench prof" bash scripts/repro_final.sh'
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/${FINAL_TAG:-final}; mkdir -p $O $ROOT/gpurun_out/final_pmc
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
PARTS=" ${PARTS:-tests pmc bench prof} "
has() { case "$PARTS" in *" $1 "*) return 0;; *) return 1;; esac; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if has pmc; then
  for wp in "sw_local 1000000" "pairhmm 100000" "semi 10000000" "nw_tb 100000" "sw_local_start 1000000" \
            "semi_start 10000000" "sw_local_300 1000000" "sw_local_tb 1000000" "nvbio_gotoh 262144" "semi_banded 10000000"; do
    set -- $wp
    bash $ROOT/scripts/pmc_session.sh $1 --workload $1 --parity-pairs 1000 >> $O/pmc_session.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then tail -3 $O/pmc_session.log; exit $rc; fi
    python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/pmc_$1 $1 $2 > /dev/null 2>> $O/pmc_summary.err || exit 1
    cp $ROOT/profiles/pmc_$1.json $ROOT/gpurun_out/final_pmc/
  done
  echo "pmc summaries done"
fi
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.json" 2> "$O/$name.err"
  local rc=$?
  echo "[$name] rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/$name.json | head -1)"
  if fatal $rc; then echo "fatal in $name"; exit $rc; fi
  return 0
}
if has bench; then
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py
step bench_sw_local_start 600 python bench.py --workload sw_local_start --cpu-seconds 8
step bench_sw_local_start_s1 600 python bench.py --workload sw_local_start --streams 1 --no-cpu
step bench_sw_local_tb 600 python bench.py --workload sw_local_tb --cpu-seconds 8
step bench_sw_local_300 600 python bench.py --workload sw_local_300 --no-cpu
step bench_sw_local_match2 600 python bench.py --workload sw_local --scores 2,4,6,1 --no-cpu
step bench_nw_tb 600 python bench.py --workload nw_tb --cpu-seconds 8
step bench_nw_tb_s1 600 python bench.py --workload nw_tb --streams 1 --no-cpu
step bench_nw_score 600 python bench.py --workload nw_score --no-cpu
step bench_semi 600 python bench.py --workload semi --cpu-seconds 8
step bench_semi_start 600 python bench.py --workload semi_start --no-cpu
step bench_semi_banded 600 python bench.py --workload semi_banded --no-cpu
step bench_pairhmm 600 python bench.py --workload pairhmm --cpu-seconds 8
step bench_nvbio_gotoh 600 python bench.py --workload nvbio_gotoh --no-cpu
step bench_nvbio_banded 600 python bench.py --workload nvbio_banded --no-cpu
step bench_ksw 600 python bench.py --workload ksw --no-cpu
step bench_boundary 600 python bench.py --workload boundary
fi
has prof || exit 0
cd /tmp && export TMPDIR=/tmp
for w in sw_local pairhmm semi semi_start sw_local_start sw_local_tb nw_tb; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
    python3 $ROOT/bench.py --workload $w --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_$w.json 2> $O/prof_$w.err
  rc=$?; echo "[prof $w] rc=$rc"; if fatal $rc; then exit $rc; fi
done
exit 0
