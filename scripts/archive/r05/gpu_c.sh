#!/bin/bash
# round 5, session C: WITH_START reading the forward sequences backwards (no reversed slots),
# the TAIL=QUERY class fix.  GPU tests of both, then the WITH_START bench lines (1 and
# 2 engines) and a kernel trace.  Output: gpurun_out/r05c/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05c; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "start or tail_query or multi" > $O/pytest_sel.log 2>&1
rc=$?; echo "pytest sel rc=$rc $(tail -1 $O/pytest_sel.log)"; [ $rc -eq 0 ] || exit $rc
for w in sw_local_start semi_start; do
  for s in 1 2; do
    timeout -k 10 300 python bench.py --workload $w --streams $s --no-cpu --no-e2e > $O/bench_${w}_s$s.json 2> $O/bench_${w}_s$s.err
    rc=$?; echo "bench $w s$s rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_${w}_s$s.json | head -1) $(grep -o '"mismatches": [0-9]*' $O/bench_${w}_s$s.json | head -1)"; [ $rc -eq 0 ] || exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
for w in sw_local_start semi_start; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
  python3 $ROOT/bench.py --workload $w --streams 1 --no-cpu --no-e2e --parity-pairs 20000 > $O/prof_$w.json 2> $O/prof_$w.err
rc=$?; echo "prof $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
