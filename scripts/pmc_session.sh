#!/bin/bash
# PMC passes for one bench workload (separate rocprofv3 runs; --pmc never combined with
# runtime/sys traces).  Usage: pmc_session.sh TAG [bench args...]
# Summarise afterwards (on the host): python tools/pmc_summary.py gpurun_out/pmc_TAG WORKLOAD PAIRS
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${1:-r01}; shift || true
OUT="$ROOT/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/bench.py" --steps 3 --no-cpu --no-e2e "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i rc=$rc ($pass)"
  if fatal $rc; then exit $rc; fi
done
exit 0
