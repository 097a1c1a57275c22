#!/bin/bash
# round 4, session U: PairHMM's last round on twice the lanes (scripts/r04/hmm_tail.patch built as
# lib/variants/libgasal_tail.so with -DGX_HMM_TAIL=1) against the final library; its PairHMM tests.
# Output: gpurun_out/r04u/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04u; mkdir -p $O
V=$ROOT/genomics-gpu_amd/lib/variants/libgasal_tail.so
GASALX_LIB=$V timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -k hmm --timeout 120 --timeout-method thread > $O/hmm_tests.log 2>&1
rc=$?; echo "hmm tests (tail) rc=$rc $(tail -1 $O/hmm_tests.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in 1 2; do
  for lib in base tail; do
    L=""; [ $lib = tail ] && L="GASALX_LIB=$V"
    env $L X=1 timeout -k 10 300 python bench.py --workload pairhmm --no-cpu --no-e2e --steps 10 --parity-pairs 100000 > $O/hmm_${lib}_$k.json 2> $O/hmm_${lib}_$k.err
    rc=$?; echo "$lib $k rc=$rc $(grep -o '"value": [0-9.]*' $O/hmm_${lib}_$k.json) $(grep -o '"mismatches": [0-9]*' $O/hmm_${lib}_$k.json | head -1)"
    [ $rc -eq 0 ] || { tail -5 $O/hmm_${lib}_$k.err; exit $rc; }
  done
done
exit 0
