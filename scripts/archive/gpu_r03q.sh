#!/bin/bash
# Round 3: ksw16 memory traffic (PMC FETCH_SIZE / WRITE_SIZE / VALU) at 1 M pairs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$ROOT/gpurun_out/r03q
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$O/p$i" -o run -- python3 "$ROOT/tools/path_probe.py" 1000000 ksw > "$O/p$i.out" 2> "$O/p$i.err"
  rc=$?; echo "pass $i rc=$rc"
  if fatal $rc; then exit $rc; fi
done
exit 0
