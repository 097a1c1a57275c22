#!/bin/bash
# A/B of library build variants (genomics-gpu_amd/lib/variants/libgasal_<name>.so via GASALX_LIB)
# on one bench workload: variant_ab.sh TAG WORKLOAD name...   ("base" = the default library)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=$1; W=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
for v in "$@" "$@"; do
  lib=""; [ "$v" != base ] && lib="GASALX_LIB=$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"
  env $lib timeout -k 10 300 python bench.py --workload $W --steps 10 --no-cpu --no-e2e --parity-pairs 20000 > "$O/$v.json" 2> "$O/$v.err" || exit $?
  python -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'])"
done
