#!/bin/bash
# round 4, session A: band traceback diagnostics, GLOBAL/TB + window-edge + packed-input +
# WITH_START parity tests, VALU issue micro-benchmark.  Output: gpurun_out/r04a/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04a; mkdir -p $O
step() {  # name timeout cmd...: run, report, stop the session on failure
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log)"
  [ $rc -eq 0 ] || { tail -40 $O/$name.log; exit $rc; }
}
PYT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread"
step ubench 120 ./tools/ubench_issue
cp $O/ubench.log $O/ubench_issue.json
step diag1 300 python -u tools/band_diag.py 8 64 600
grep -v amdgpu.ids $O/diag1.log | tail -20
step diag2 300 python -u tools/band_diag.py 20 310 700
grep -v amdgpu.ids $O/diag2.log | tail -20
step tbtests 600 $PYT tests/test_gpu_parity.py -k "global or kat or config3 or traceback"
step edges 900 $PYT tests/test_gpu_window_edges.py
step packed 300 $PYT tests/test_gpu_parity.py -k "packed_input"
step start 600 $PYT tests/test_gpu_parity.py -k "with_start or start"
exit 0
