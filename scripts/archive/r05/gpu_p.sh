#!/bin/bash
# round 5, session P: the band walk's diagonal chunk and code-block prefetch (generic.hpp tb_kernel)
# against HEAD's library (lib/variants/libgasal_base.so, commit d89d399): the traceback GPU tests,
# then config 3 on one and three engines, alternating, and a one-engine trace of each.
# Output: gpurun_out/r05p/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "traceback or config3 or tb or cigar" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
V=$ROOT/genomics-gpu_amd/lib/variants/libgasal_base.so
for k in 1 2; do
  for s in 1 3; do
    for lib in new base; do
      E="GASALX_DUMMY=1"; [ $lib = base ] && E="GASALX_LIB=$V"
      env $E timeout -k 10 300 python bench.py --workload nw_tb --streams $s --no-cpu --no-e2e --parity-pairs 20000 > $O/nw_tb_s${s}_${lib}_$k.json 2> $O/nw_tb_s${s}_${lib}_$k.err
      rc=$?; echo "nw_tb s$s $lib $k rc=$rc $(grep -o '"value": [0-9.]*' $O/nw_tb_s${s}_${lib}_$k.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/nw_tb_s${s}_${lib}_$k.json | head -1)"
      [ $rc -eq 0 ] || { tail -3 $O/nw_tb_s${s}_${lib}_$k.err; exit $rc; }
    done
  done
done
for lib in new base; do
  E="GASALX_DUMMY=1"; [ $lib = base ] && E="GASALX_LIB=$V"
  (cd /tmp && export TMPDIR=/tmp && env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- \
    python3 $ROOT/bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_$lib.json 2> $O/prof_$lib.err)
  echo "prof $lib rc=$?"
done
exit 0
