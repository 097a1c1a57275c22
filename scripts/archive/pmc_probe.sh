#!/bin/bash
# PMC passes over tools/path_probe.py for one mode: pmc_probe.sh MODE [pairs]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
M=$1; N=${2:-200000}
OUT="$ROOT/gpurun_out/pmcp_$M"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$OUT/p$i" -o run -- python3 "$ROOT/tools/path_probe.py" $N $M > "$OUT/p$i.out" 2> "$OUT/p$i.err"
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
