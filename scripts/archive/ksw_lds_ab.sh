#!/bin/bash
# KSW: parity tests, then the path probe's ksw line with the level-0 entries in LDS
# (default) and in the global [column][pair] array (GASALX_KSW_LDS=0)
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=gpurun_out/ksw_lds; mkdir -p "$O"
bash scripts/gpu_quick.sh ksw_tests "ksw" || exit $?
for n in 200000 1000000; do
  for v in 1 0 1; do
    GASALX_KSW_LDS=$v timeout -k 10 300 python tools/path_probe.py $n ksw > "$O/p${v}_$n.jsonl" 2> "$O/p${v}_$n.err" || exit $?
    echo "lds=$v $(tail -1 "$O/p${v}_$n.jsonl")"
  done
done
