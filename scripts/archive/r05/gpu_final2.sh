#!/bin/bash
# round 5, final library (band half width 22): the full GPU suite, then the PMC passes of every
# bench workload (summarised on the host into profiles/pmc_*.json), all in one call.
# Output: gpurun_out/r05final2/, gpurun_out/pmc_<workload>/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05final2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash $ROOT/scripts/r05/gpu_pmc.sh
