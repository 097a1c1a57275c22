#!/bin/bash
# Timing probe of the GLOBAL+TB direction stores (GX_TB_STORE_MODE variants; results of
# the probes are invalid by design): rocprof kernel stats of config 3 per variant.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$ROOT/gpurun_out/${1:-tbstore}; shift; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib=""; [ "$v" != base ] && lib=$ROOT/genomics-gpu_amd/lib/variants/libgasal_$v.so
  GASALX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$v" -o run -- python3 "$ROOT/bench.py" --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > "$O/$v.out" 2> "$O/$v.err"
  rc=$?; echo "[$v] rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
  grep -h "wf16\|tb_kernel" "$O/prof_$v/run_kernel_stats.csv" | cut -d, -f1-4
done
