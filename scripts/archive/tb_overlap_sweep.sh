#!/bin/bash
# GPU parity tests, then the DP + traceback-walk overlap chunk count (GASALX_TB_CHUNKS)
# on the two traceback workloads.  Stops at the first fatal exit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out/${1:-s4}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/t.out" 2>&1
rc=$?
tail -3 "$O/t.out"
grep -E "^E " "$O/t.out" | head -5
[ $rc -eq 0 ] || exit $rc
for k in 1 2 4 8; do
  for w in nw_tb sw_local_tb; do
    GASALX_TB_CHUNKS=$k timeout -k 10 300 python bench.py --workload $w --steps 10 --no-cpu --no-e2e > "$O/b_${w}_$k.json" || exit $?
    echo "chunks=$k $w $(cut -c1-160 "$O/b_${w}_$k.json")"
  done
done
exit 0
