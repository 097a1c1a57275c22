#!/bin/bash
# Round 3: drift LOCAL WITH_START mismatch triage.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ah; mkdir -p $O
GASALX_KF16=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -m gpu -q --timeout 120 --timeout-method thread -k "traceback_and_start" > $O/kf0.log 2>&1
echo "kf0 rc=$? $(tail -1 $O/kf0.log)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -k "local or start" > $O/kf1.log 2>&1
echo "kf1 rc=$? $(tail -1 $O/kf1.log)"
timeout -k 10 300 python tools/drift_triage.py > $O/triage.txt 2>&1
echo "triage rc=$?"
