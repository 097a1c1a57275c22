#!/bin/bash
# Round 3: the packed (two pairs per lane) nvbio banded kernel: GPU parity, A/B bench, kernel stats.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$ROOT/gpurun_out/r03t
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_nvbio.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --workload nvbio_banded --steps 10 --warmup 3 > $O/bench16.json 2> $O/bench16.err
rc=$?; echo "bench16 rc=$rc $(tail -1 $O/bench16.json)"; [ $rc -eq 0 ] || exit $rc
GASALX_NVB16=0 timeout -k 10 240 python bench.py --workload nvbio_banded --steps 10 --warmup 3 --no-cpu --no-e2e > $O/bench32.json 2> $O/bench32.err
rc=$?; echo "bench32 rc=$rc $(tail -1 $O/bench32.json)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$ROOT/bench.py" --workload nvbio_banded --steps 5 --warmup 2 --no-cpu --no-e2e > $O/prof.out 2> $O/prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
