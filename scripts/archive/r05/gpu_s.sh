#!/bin/bash
# round 5, session S: the striped nvbio traceback kernel: its GPU tests, then the throughput probe.
# Output: gpurun_out/r05s/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_nvbio.py -x -q --timeout 120 --timeout-method thread -k traceback > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/nv_traceback_probe.py 65536 32 > $O/probe.jsonl 2> $O/probe.err
rc=$?; cat $O/probe.jsonl; [ $rc -eq 0 ] || { tail -5 $O/probe.err; exit $rc; }
