#!/bin/bash
# round 5, session R: throughput of the nvbio traceback front-end (tools/nv_traceback_probe.py) and a
# kernel trace of it.  Output: gpurun_out/r05r/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python tools/nv_traceback_probe.py 65536 32 > $O/probe.jsonl 2> $O/probe.err
rc=$?; cat $O/probe.jsonl; [ $rc -eq 0 ] || { tail -5 $O/probe.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $ROOT/tools/nv_traceback_probe.py 16384 32 > $O/prof.jsonl 2> $O/prof.err
echo "prof rc=$?"
