#!/bin/bash
# banded: parity tests, then the semi_banded bench with the packed kernel and with the int32 kernel only
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/band; mkdir -p "$O"
bash scripts/gpu_quick.sh band_tests "banded" || exit $?
for v in 1 0 1; do
  GASALX_BAND16=$v timeout -k 10 300 python bench.py --workload semi_banded --steps 10 --no-cpu --no-e2e --parity-pairs 200000 > "$O/b$v.json" 2> "$O/b$v.err" || exit $?
  python -c "import json; d=json.loads(open('$O/b$v.json').read().strip().splitlines()[-1]); print('band16=$v', d['config']['plan'], d['value'], d['ms_per_step'], d['parity'])"
done
