#!/bin/bash
# round 5, session M: config 2 on the G16R10 shape (GASALX_GMIN=16: 4 waves per SIMD, 99 VGPRs,
# 2x the lanes per pair) against the default G8R19 (3 waves per SIMD, LDS-bound), alternating.
# Output: gpurun_out/r05m/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05m; mkdir -p $O
for k in 1 2; do
  for v in g8 g16; do
    E="GASALX_DUMMY=1"; [ $v = g16 ] && E="GASALX_GMIN=16"
    env $E timeout -k 10 300 python bench.py --workload sw_local --no-cpu --no-e2e --parity-pairs 20000 > $O/sw_local_${v}_$k.json 2> $O/sw_local_${v}_$k.err
    rc=$?; echo "sw_local $v $k rc=$rc $(grep -o '"value": [0-9.]*' $O/sw_local_${v}_$k.json | head -1) $(grep -o '"plan": "[^"]*"' $O/sw_local_${v}_$k.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/sw_local_${v}_$k.json | head -1)"
    [ $rc -eq 0 ] || { tail -3 $O/sw_local_${v}_$k.err; exit $rc; }
  done
done
exit 0
