#!/bin/bash
# Round 3: nvbio BatchedBandedAlignmentScore front-end: GPU parity + bench line + kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03k
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_nvbio.py -x -q --timeout 300 --timeout-method thread > $O/nv.txt 2>&1
rc=$?; echo "nvbio tests rc=$rc"; tail -3 $O/nv.txt; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload nvbio_banded --steps 10 --warmup 2 --no-e2e --parity-pairs 200000 > $O/banded.json 2> $O/banded.err
rc=$?; echo "nvbio_banded rc=$rc $(python -c "import json;d=json.load(open('$O/banded.json'));print(d['value'],d['parity'])" 2>/dev/null)"
if fatal $rc; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload nvbio_banded --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > $GRAFT_REPO_ROOT/$O/prof.json 2>&1
echo "prof rc=$?"
exit 0
