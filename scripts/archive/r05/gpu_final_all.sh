#!/bin/bash
# round 5, the last library, in one call: the full GPU suite, the PMC passes of every bench workload
# summarised on the box (tools/pmc_summary.py, so the bench lines after them carry the traffic and
# issue-priced figures of this same library; copies under gpurun_out/final_pmc/), then every bench
# line and the kernel traces (scripts/r05/gpu_final.sh).  Output: gpurun_out/${FINAL_TAG}/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
export FINAL_TAG=${FINAL_TAG:-r05final5}
O=$ROOT/gpurun_out/$FINAL_TAG; mkdir -p $O $ROOT/gpurun_out/final_pmc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
PMC_WORKLOADS="sw_local pairhmm semi nw_tb sw_local_start semi_start sw_local_300 sw_local_tb nvbio_gotoh semi_banded" \
  bash $ROOT/scripts/r05/gpu_pmc.sh > $O/pmc_session.log 2>&1 || { tail -3 $O/pmc_session.log; exit 1; }
for wp in "sw_local 1000000" "pairhmm 100000" "semi 10000000" "nw_tb 100000" "sw_local_start 1000000" \
          "semi_start 10000000" "sw_local_300 1000000" "sw_local_tb 1000000" "nvbio_gotoh 262144" "semi_banded 10000000"; do
  set -- $wp
  python3 $ROOT/tools/pmc_summary.py $ROOT/gpurun_out/pmc_$1 $1 $2 > /dev/null 2>> $O/pmc_summary.err || exit 1
  cp $ROOT/profiles/pmc_$1.json $ROOT/gpurun_out/final_pmc/
done
echo "pmc summaries done"
bash $ROOT/scripts/r05/gpu_final.sh
