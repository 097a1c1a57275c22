#!/bin/bash
# LOCAL second best: parity tests, then the path probe's local_second line with the
# packed kernel (GASALX_LOCAL16 unset) and with the int32 kernel only
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/local16; mkdir -p "$O"
bash scripts/gpu_quick.sh local16_tests "local16 or second" || exit $?
for v in 1 0 1; do
  GASALX_LOCAL16=$v timeout -k 10 300 python tools/path_probe.py 200000 local_second > "$O/p$v.jsonl" 2> "$O/p$v.err" || exit $?
  echo "local16=$v $(tail -1 "$O/p$v.jsonl")"
done
