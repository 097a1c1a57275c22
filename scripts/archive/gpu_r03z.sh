#!/bin/bash
# Round 3 (re-entry): headline + config 3 + config 5 bench lines at the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03z
mkdir -p $O
for w in sw_local nw_tb pairhmm; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --cpu-seconds 5 > $O/bench_$w.json 2> $O/bench_$w.err
  rc=$?; echo "$w rc=$rc"; tail -c 600 $O/bench_$w.json; [ $rc -eq 0 ] || exit $rc
done
