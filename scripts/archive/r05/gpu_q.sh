#!/bin/bash
# round 5, session Q: the nvbio BatchedAlignmentTraceback front-end (nvtrace.hpp): its GPU tests
# and the rest of the nvbio suite.  Output: gpurun_out/r05q/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_nvbio.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; exit $rc
