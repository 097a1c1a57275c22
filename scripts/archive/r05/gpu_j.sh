#!/bin/bash
# round 5, session J: this tree (kernel body as wf16_body.inc, rclass reverse passes, two-phase
# SEMI sweep) against HEAD's library (lib/variants/libgasal_base.so) on every main workload,
# alternating, then one-engine kernel traces of semi and semi_start.  Output: gpurun_out/r05j/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05j; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
V=$ROOT/genomics-gpu_amd/lib/variants/libgasal_base.so
for k in 1 2; do
  for w in semi semi_start sw_local_start sw_local nw_tb; do
    for lib in new base; do
      E="GASALX_DUMMY=1"; [ $lib = base ] && E="GASALX_LIB=$V"
      env $E timeout -k 10 300 python bench.py --workload $w --no-cpu --no-e2e --parity-pairs 20000 > $O/${w}_${lib}_$k.json 2> $O/${w}_${lib}_$k.err
      rc=$?; echo "$w $lib $k rc=$rc $(grep -o '"value": [0-9.]*' $O/${w}_${lib}_$k.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/${w}_${lib}_$k.json | head -1)"
      [ $rc -eq 0 ] || { tail -3 $O/${w}_${lib}_$k.err; exit $rc; }
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for w in semi semi_start; do
  for lib in new base; do
    if [ $lib = base ]; then export GASALX_LIB=$V; else unset GASALX_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${w}_$lib -o run -- \
      python3 $ROOT/bench.py --workload $w --streams 1 --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_${w}_$lib.json 2> $O/prof_${w}_$lib.err
    rc=$?; echo "prof $w $lib rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
