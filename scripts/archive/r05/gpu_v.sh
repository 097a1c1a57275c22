#!/bin/bash
# round 5, session V: run-to-run spread on one box of the final library: the default (headline)
# line five times, config 3 (three engines) three times.  Output: gpurun_out/r05v/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05v; mkdir -p $O
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu --no-e2e > $O/default_$r.json 2> $O/default_$r.err || exit $?
  grep -o '"value": [0-9.]*' $O/default_$r.json
done
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --workload nw_tb --no-cpu --no-e2e > $O/nw_tb_$r.json 2> $O/nw_tb_$r.err || exit $?
  grep -o '"value": [0-9.]*' $O/nw_tb_$r.json
done
