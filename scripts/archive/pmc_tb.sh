#!/bin/bash
# PMC passes over config 3 (nw_tb) for the walk kernel: where tb_kernel's time goes.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/pmc_tb"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/bench.py" --workload nw_tb --steps 3 --warmup 1 --no-cpu --no-e2e --parity-pairs 0 > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
exit 0
