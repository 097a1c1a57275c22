#!/bin/bash
# round 5, session N3: config 3 (band widths around the fallback-free one)'s band half width w (GASALX_TB_BAND_W) on one engine and on three,
# alternating; the one-engine chain carries the fallback's latency floor whenever a pair leaves the
# band.  Output: gpurun_out/r05n3/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05n3; mkdir -p $O
for k in 1 2; do
  for s in 1 3; do
    for w in 22 24 26 28; do
      GASALX_TB_BAND_W=$w timeout -k 10 300 python bench.py --workload nw_tb --streams $s --no-cpu --no-e2e --parity-pairs 20000 > $O/nw_tb_s${s}_w${w}_$k.json 2> $O/nw_tb_s${s}_w${w}_$k.err
      rc=$?; echo "nw_tb s$s w$w $k rc=$rc $(grep -o '"value": [0-9.]*' $O/nw_tb_s${s}_w${w}_$k.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/nw_tb_s${s}_w${w}_$k.json | head -1)"
      [ $rc -eq 0 ] || { tail -3 $O/nw_tb_s${s}_w${w}_$k.err; exit $rc; }
    done
  done
done
exit 0
