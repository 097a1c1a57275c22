#!/bin/bash
# round 4, session O: the full GPU test suite on the final library, then the final bench lines of the
# remaining workloads (scripts/r04/gpu_n.sh without the profiling pass).
# Output: gpurun_out/r04o/, gpurun_out/r04final/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"
[ $rc -eq 0 ] || { grep -E "^FAILED|^ERROR|Error" $O/gpu_tests.log | head -20; [ $rc -eq 1 ] || exit $rc; }
SKIP_PROF=1 WORKLOADS="${WORKLOADS:-sw_local_start semi_start semi_banded nvbio_gotoh nvbio_banded ksw nw_score cpu_plumbing}" bash $ROOT/scripts/r04/gpu_n.sh
