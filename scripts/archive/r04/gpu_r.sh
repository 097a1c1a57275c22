#!/bin/bash
# round 4, session R: PairHMM with the staged bytes masked to their code bits (GX_HMM_MASKB, variant
# library) against the final library; config 3's band half width with three engines.
# Output: gpurun_out/r04r/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04r; mkdir -p $O
run() {
  local name=$1 envs=$2 w=$3; shift 3
  env $envs timeout -k 10 300 python bench.py --workload $w --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json) $(grep -o '"mismatches": [0-9]*' $O/$name.json | head -1)"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
V=$ROOT/genomics-gpu_amd/lib/variants
run hmm_base "X=1" pairhmm --steps 10 --parity-pairs 100000
run hmm_maskb "GASALX_LIB=$V/libgasal_maskb.so" pairhmm --steps 10 --parity-pairs 100000
run hmm_base2 "X=1" pairhmm --steps 10 --parity-pairs 1000
run hmm_maskb2 "GASALX_LIB=$V/libgasal_maskb.so" pairhmm --steps 10 --parity-pairs 1000
GASALX_LIB=$V/libgasal_maskb.so timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -k hmm --timeout 120 --timeout-method thread > $O/hmm_tests_maskb.log 2>&1
echo "maskb hmm tests rc=$? $(tail -1 $O/hmm_tests_maskb.log)"
for w in 8 10 12; do run nw_tb_w$w "GASALX_TB_BAND_W=$w" nw_tb --steps 12 --parity-pairs 100000; done
exit 0
