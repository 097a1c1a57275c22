#!/bin/bash
# A/B of the PairHMM column-update variants (GASALX_HMM_VARIANT, GASALX_HMM_RR16; pairhmm.hpp) on config 5.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/${1:-hmm_ab}; mkdir -p "$O"
for cfg in ${CFGS:-0 1 0r 1r}; do
  v=${cfg%r}; rr=""; [ "$cfg" != "$v" ] && rr=1
  env GASALX_HMM_VARIANT=$v ${rr:+GASALX_HMM_RR16=1} timeout -k 10 300 python bench.py --workload pairhmm --steps 10 --no-cpu --no-e2e --parity-pairs 20000 > "$O/$cfg.json" 2> "$O/$cfg.err" || exit $?
  python -c "import json,sys; d=json.loads(open('$O/$cfg.json').read().strip().splitlines()[-1]); print('cfg $cfg', d['value'], d['ms_per_step'], d['parity']['mismatches'])"
done
