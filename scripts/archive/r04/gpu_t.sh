#!/bin/bash
# round 4, session T: three engines for the WITH_START workloads.
# Output: gpurun_out/r04t/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04t; mkdir -p $O
run() {
  local name=$1 w=$2; shift 2
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json) $(grep -o '"mismatches": [0-9]*' $O/$name.json | head -1)"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
}
run start_s2 sw_local_start --steps 6 --parity-pairs 100000 --streams 2
run start_s3 sw_local_start --steps 6 --parity-pairs 100000 --streams 3
run semi_start_s2 semi_start --steps 4 --parity-pairs 100000 --streams 2
run semi_start_s3 semi_start --steps 6 --parity-pairs 100000 --streams 3
run ltb_s1 sw_local_tb --steps 6 --parity-pairs 100000 --streams 1
run ltb_s2 sw_local_tb --steps 6 --parity-pairs 100000 --streams 2
exit 0
