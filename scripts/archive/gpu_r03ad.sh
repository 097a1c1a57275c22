#!/bin/bash
# Round 3: LOCAL timing probes (results invalid by construction): which extension
# subtract bounds the headline kernel.  base / pf (F) / pe (E) / pfe (both).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ad; mkdir -p $O
for v in base pf pe pfe base pf pe pfe; do
  lib=""; [ "$v" != base ] && lib="GASALX_LIB=$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"
  env $lib timeout -k 10 300 python bench.py --steps 10 --no-cpu --no-e2e --parity-pairs 2000 > "$O/$v.json" 2> "$O/$v.err"
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
  python -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'])"
done
