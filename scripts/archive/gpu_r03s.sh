#!/bin/bash
# Round 3: are the strip-walking packed kernels (local16 second best, banded16) HBM-bound?
# PMC FETCH / WRITE / VALU passes on the path probe at 1 M pairs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$ROOT/gpurun_out/r03s
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp
for mode in local_second banded16; do
  i=0
  for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pass --output-format csv -d "$O/${mode}_p$i" -o run -- python3 "$ROOT/tools/path_probe.py" 1000000 $mode > "$O/${mode}_p$i.out" 2> "$O/${mode}_p$i.err"
    rc=$?; echo "$mode pass $i rc=$rc $(tail -1 $O/${mode}_p$i.out)"
    if fatal $rc; then exit $rc; fi
  done
done
exit 0
