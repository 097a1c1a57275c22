#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04band2; mkdir -p $O
timeout -k 10 300 python -u tools/band_diag.py 8 64 600 > $O/diag1.log 2>&1; rc=$?; cat $O/diag1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_diag.py 20 310 700 > $O/diag2.log 2>&1; rc=$?; cat $O/diag2.log; [ $rc -eq 0 ] || exit $rc
