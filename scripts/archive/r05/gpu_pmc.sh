#!/bin/bash
# round 5, final library: the PMC passes of every bench workload (scripts/pmc_session.sh, separate
# rocprofv3 --pmc runs, no traces combined), summarised on the host afterwards with
# tools/pmc_summary.py into profiles/pmc_<workload>.json.  Output: gpurun_out/pmc_<workload>/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
for w in ${PMC_WORKLOADS:-sw_local pairhmm semi nw_tb sw_local_start semi_start sw_local_300 sw_local_tb}; do
  bash "$ROOT/scripts/pmc_session.sh" "$w" --workload "$w" --parity-pairs 1000 || exit $?
done
exit 0
