#!/bin/bash
# Round 3: step_semi with the shorter dependency chain (GX_SEMI_CHAIN2 variant) against
# the default library, config 4, parity on the first 200 K timed pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03am; mkdir -p $O
for v in base sc2 base sc2; do
  lib=""; [ "$v" != base ] && lib="GASALX_LIB=$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"
  env $lib timeout -k 10 300 python bench.py --workload semi --steps 10 --no-cpu --no-e2e --parity-pairs 200000 > "$O/$v.json" 2> "$O/$v.err"
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'])"
done
