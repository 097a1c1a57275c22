#!/bin/bash
# round 4, session I: kernel-trace summaries (config 3 fused band, config 2 + start, config 4)
# and the config-4 / config-3 HBM counters.  Output: gpurun_out/r04i/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/r04i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() {  # name env bench-args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 $ROOT/bench.py --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
  f=$(find $O/$name -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:9]:
    print("   %-70s calls %5s avg %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
}
pmc() {  # name counters bench-args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/$name -o run -- \
    python3 $ROOT/bench.py --no-cpu --no-e2e --steps 2 --warmup 1 "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
prof nw_tb_s1 "X=1" --workload nw_tb --steps 5 --warmup 1 --streams 1 --parity-pairs 20000
prof start "X=1" --workload sw_local_start --steps 5 --warmup 1 --parity-pairs 20000
prof semi "X=1" --workload semi --steps 3 --warmup 1 --parity-pairs 20000
pmc semi_fetch FETCH_SIZE --workload semi --parity-pairs 1000
pmc semi_write WRITE_SIZE --workload semi --parity-pairs 1000
pmc nwtb_fetch FETCH_SIZE --workload nw_tb --streams 1 --parity-pairs 1000
pmc nwtb_write WRITE_SIZE --workload nw_tb --streams 1 --parity-pairs 1000
exit 0
