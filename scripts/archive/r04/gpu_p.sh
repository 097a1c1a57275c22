#!/bin/bash
# round 4, session P: engines per GPU.  The reference's test_prog drives NB_STREAMS = 2 storages per
# host thread (test_prog.cpp:12,205), one per stream; a call's kernels run in order on its stream,
# so the small kernels between a call's big ones (WITH_START: reverse-pass prep; TB: walks, fallback)
# leave the GPU partly idle unless another engine's kernels fill it.
# Output: gpurun_out/r04p/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04p; mkdir -p $O
run() {
  local name=$1 w=$2; shift 2
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json) $(grep -o '"mismatches": [0-9]*' $O/$name.json | head -1)"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run start_s1 sw_local_start --steps 6 --parity-pairs 100000 --streams 1
run start_s2 sw_local_start --steps 6 --parity-pairs 100000 --streams 2
run nw_tb_s2 nw_tb --steps 10 --parity-pairs 100000 --streams 2
run nw_tb_s3 nw_tb --steps 12 --parity-pairs 100000 --streams 3
run nw_tb_s4 nw_tb --steps 12 --parity-pairs 100000 --streams 4
run ltb_s3 sw_local_tb --steps 6 --parity-pairs 100000 --streams 3
run semi_start_s2 semi_start --steps 4 --parity-pairs 100000 --streams 2
exit 0
