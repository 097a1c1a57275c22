#!/bin/bash
# round 4, session N: the final library (walk as before, vector CIGAR-buffer copy, fenced PairHMM
# prefetch): the final rocprofv3 + PMC pass, its PMC summaries, then the final bench lines of the
# workloads in WORKLOADS (bench.py reads profiles/pmc_<w>.json of the same library).
# Output: gpurun_out/r04final/, gpurun_out/pmc_<w>/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
if [ "${SKIP_PROF:-0}" != 1 ]; then
  bash $ROOT/scripts/r04/final_prof.sh || exit $?
fi
cd $ROOT
for w in "sw_local 1000000" "semi 10000000" "nw_tb 100000" "pairhmm 100000" "sw_local_300 1000000"; do
  set -- $w
  [ -d gpurun_out/pmc_$1 ] && python3 tools/pmc_summary.py gpurun_out/pmc_$1 $1 $2 > /dev/null
done
bash $ROOT/scripts/r04/final_bench.sh
