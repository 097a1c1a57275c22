#!/bin/bash
# PMC passes for every bench workload, one after the other (stops on a fatal exit).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for w in sw_local semi nw_tb pairhmm; do
  bash "$ROOT/scripts/pmc_session.sh" "$w" --workload "$w" || exit $?
done
exit 0
