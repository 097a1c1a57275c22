#!/bin/bash
# round 5, session F: same-box A/B of this round's library against round 4's (GASALX_LIB=
# lib/variants/libgasal_r04.so, built from commit 60a0d36), two alternations per workload, then a
# kernel trace of each for the headline and PairHMM.  Output: gpurun_out/r05f/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05f; mkdir -p $O
V=$ROOT/genomics-gpu_amd/lib/variants/libgasal_r04.so
for w in sw_local pairhmm semi nw_tb sw_local_start; do
  for k in 1 2; do
    for lib in new r04; do
      L=""; [ $lib = r04 ] && L="GASALX_LIB=$V"
      env $L timeout -k 10 300 python bench.py --workload $w --no-cpu --no-e2e --parity-pairs 20000 > $O/${w}_${lib}_$k.json 2> $O/${w}_${lib}_$k.err
      rc=$?; echo "$w $lib $k rc=$rc $(grep -o '"value": [0-9.]*' $O/${w}_${lib}_$k.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/${w}_${lib}_$k.json | head -1)"
      [ $rc -eq 0 ] || { tail -3 $O/${w}_${lib}_$k.err; exit $rc; }
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for w in sw_local pairhmm; do
  for lib in new r04; do
    L=""; [ $lib = r04 ] && L="GASALX_LIB=$V"
    env $L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${w}_$lib -o run -- \
      python3 $ROOT/bench.py --workload $w --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_${w}_$lib.json 2> $O/prof_${w}_$lib.err
    rc=$?; echo "prof $w $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
