#!/bin/bash
# round 5, session G: the register-axis class kernels of the WITH_START reverse passes
# (rclass.hip) and the phased SEMI sweep.  GPU tests of the start / semi paths, then same-box
# A/B benches: this tree's library, the same with GASALX_RCLASS=0, and HEAD's library
# (lib/variants/libgasal_base.so, commit 4cfd6e2).  Output: gpurun_out/r05g/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "start or semi or Start or SEMI" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
V=$ROOT/genomics-gpu_amd/lib/variants/libgasal_base.so
run() {  # name env... -- bench args
  local name=$1; shift
  env "$@" > $O/$name.json 2> $O/$name.err
}
for k in 1 2; do
  for w in semi_start sw_local_start semi; do
    for lib in new norc base; do
      [ $w = semi ] && [ $lib = norc ] && continue
      E="GASALX_DUMMY=1"; [ $lib = norc ] && E="GASALX_RCLASS=0"; [ $lib = base ] && E="GASALX_LIB=$V"
      X=""; [ $w = sw_local_start ] && X="--streams 1"
      env $E timeout -k 10 300 python bench.py --workload $w $X --no-cpu --no-e2e --parity-pairs 20000 > $O/${w}_${lib}_$k.json 2> $O/${w}_${lib}_$k.err
      rc=$?; echo "$w $lib $k rc=$rc $(grep -o '"value": [0-9.]*' $O/${w}_${lib}_$k.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/${w}_${lib}_$k.json | head -1)"
      [ $rc -eq 0 ] || { tail -3 $O/${w}_${lib}_$k.err; exit $rc; }
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_semi_start -o run -- \
  python3 $ROOT/bench.py --workload semi_start --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_semi_start.json 2> $O/prof_semi_start.err
echo "prof rc=$?"
exit 0
