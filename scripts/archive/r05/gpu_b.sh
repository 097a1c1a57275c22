#!/bin/bash
# round 5, session B: the time-based warmup.  Bench lines (sw_local, pairhmm) with the default
# warmup, each beside a rocprofv3 kernel trace of the same command; and the clock ramp of a cold
# GPU: pairhmm with no warmup, 60 traced steps.  Output: gpurun_out/r05b/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/r05b; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ramp -o run -- \
  python3 $ROOT/bench.py --workload pairhmm --no-cpu --no-e2e --warmup 0 --steps 60 --parity-pairs 1000 > $O/ramp.json 2> $O/ramp.err
rc=$?; echo "ramp rc=$rc"; [ $rc -eq 0 ] || exit $rc
for w in sw_local pairhmm nw_tb; do
  timeout -k 10 300 python3 $ROOT/bench.py --workload $w --no-cpu --no-e2e > $O/bench_$w.json 2> $O/bench_$w.err
  rc=$?; echo "bench $w rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_$w.json | head -1) $(grep -o '"warmup": [0-9]*' $O/bench_$w.json)"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
    python3 $ROOT/bench.py --workload $w --no-cpu --no-e2e > $O/prof_$w.json 2> $O/prof_$w.err
  rc=$?; echo "prof $w rc=$rc $(grep -o '"value": [0-9.]*' $O/prof_$w.json | head -1)"; [ $rc -eq 0 ] || exit $rc
done
exit 0
