#!/bin/bash
# GPU parity tests, then kernel time at the reference's own batch size (5,000 pairs)
# and at 20,000 / 1M pairs of its sample data, and the headline bench.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out/${1:-small}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/t.out" 2>&1
rc=$?; tail -2 "$O/t.out"; grep -E "^E " "$O/t.out" | head -5
[ $rc -eq 0 ] || exit $rc
for n in 5000 20000 1000000; do
  timeout -k 10 300 python tools/sample_probe.py $n local,semi_tt,global > "$O/p_$n.out" 2>&1 || exit $?
  grep mode "$O/p_$n.out" | cut -c1-200
done
timeout -k 10 300 python bench.py --no-cpu --no-e2e --steps 10 > "$O/bench.json" || exit $?
cut -c1-200 "$O/bench.json"
exit 0
