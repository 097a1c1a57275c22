#!/bin/bash
# round 5, session U: rocprofv3 kernel trace and HBM counters (separate passes) of the nvbio
# traceback probe on the final library.  Output: gpurun_out/r05u/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/r05u; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $ROOT/tools/nv_traceback_probe.py 262144 32 > $O/trace.jsonl 2> $O/trace.err || exit $?
echo "[trace] ok"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- \
  python3 $ROOT/tools/nv_traceback_probe.py 262144 32 > $O/fetch.jsonl 2> $O/fetch.err || exit $?
echo "[fetch] ok"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- \
  python3 $ROOT/tools/nv_traceback_probe.py 262144 32 > $O/write.jsonl 2> $O/write.err || exit $?
echo "[write] ok"
