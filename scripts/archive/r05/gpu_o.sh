#!/bin/bash
# round 5, session O: one-engine kernel trace of config 3 (band half width 22), to price the chain
# around the fused kernel.  Output: gpurun_out/r05o/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/r05o; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nw_tb_s1 -o run -- \
  python3 $ROOT/bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_nw_tb_s1.json 2> $O/prof_nw_tb_s1.err
echo "prof rc=$?"
