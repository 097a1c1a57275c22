#!/bin/bash
# Round 3: packed nvbio banded kernel with band-length instances (8/16/32 exact) and the
# row's F first: nvbio GPU tests, bench nvbio_banded (2 runs), kernel stats.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$ROOT/gpurun_out/r03x
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_nvbio.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 240 python bench.py --workload nvbio_banded --steps 10 --warmup 3 --no-cpu --no-e2e > $O/bench_$rep.json 2> $O/bench_$rep.err
  rc=$?; echo "bench rc=$rc $(python -c "import json;d=json.load(open('$O/bench_$rep.json'));print(d['value'],d['roofline']['kernel_ms'],d['parity']['mismatches'])")"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$ROOT/bench.py" --workload nvbio_banded --steps 5 --warmup 2 --no-cpu --no-e2e > $O/prof.out 2> $O/prof.err
rc=$?; echo "prof rc=$rc"; exit $rc
