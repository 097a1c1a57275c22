#!/bin/bash
# GPU parity tests, then the reference's sample data with and without the length sort.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out/${1:-sort}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/t.out" 2>&1
rc=$?; tail -2 "$O/t.out"; grep -E "^E " "$O/t.out" | head -5
[ $rc -eq 0 ] || exit $rc
for srt in 0 1; do
  GASALX_SORT=$srt timeout -k 10 300 python tools/sample_probe.py 1000000 > "$O/p_$srt.out" 2>&1 || exit $?
  grep mode "$O/p_$srt.out"
done
exit 0
