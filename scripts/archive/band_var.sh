#!/bin/bash
# banded bench across library variants (GASALX_LIB): band_var.sh name...  ("base" = default library)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/bandvar; mkdir -p "$O"
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib="GASALX_LIB=$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"
  env $lib timeout -k 10 300 python bench.py --workload semi_banded --steps 10 --no-cpu --no-e2e --parity-pairs 100000 > "$O/$v.json" 2> "$O/$v.err" || exit $?
  python -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['config']['plan'], d['value'], d['ms_per_step'], d['parity']['mismatches'])"
done
