#!/bin/bash
# Round 3: nvbio16 Gotoh drift frame: nvbio GPU tests + nvbio_gotoh bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03af; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "nvbio" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload nvbio_gotoh --steps 10 --no-cpu > $O/bench_nvbio_gotoh.json 2> $O/bench_nvbio_gotoh.err
rc=$?; echo "nvbio_gotoh rc=$rc"; python -c "import json; d=json.loads(open('$O/bench_nvbio_gotoh.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatches'], d['config'].get('plan'))"
