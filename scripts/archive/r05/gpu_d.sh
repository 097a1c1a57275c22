#!/bin/bash
# round 5, session D: the full GPU suite on the library with the one-division strip-major merge,
# the grid-stride int32 fallback, the wave-aggregated slot sort and the in-place reverse pass; then
# the bench lines they touch.  Output: gpurun_out/r05d/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05d; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.log | head -20; exit $rc; }
for w in sw_local pairhmm sw_local_start:1 sw_local_start:2 semi_start:2 semi sw_local_tb nw_tb nw_tb:1 sw_local_300; do
  n=${w%%:*}; s=${w#*:}; [ "$s" = "$w" ] && s=""
  timeout -k 10 300 python bench.py --workload $n ${s:+--streams $s} --no-cpu --no-e2e > $O/bench_${n}${s:+_s$s}.json 2> $O/bench_${n}${s:+_s$s}.err
  rc=$?; echo "bench $w rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_${n}${s:+_s$s}.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/bench_${n}${s:+_s$s}.json | head -1)"; [ $rc -eq 0 ] || exit $rc
done
exit 0
