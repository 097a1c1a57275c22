#!/bin/bash
# Round 3 final PMC: the bench workloads whose lines carry `traffic` / `issue` (separate
# rocprofv3 --pmc passes per workload, scripts/pmc_session.sh; the timed step only:
# no parity, no host-staged timing).  Usage: pmc_r03.sh WORKLOAD...
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for w in "$@"; do
  bash "$ROOT/scripts/pmc_session.sh" "$w" --workload "$w" --parity-pairs 0 --no-e2e --streams 1 || exit $?
done
exit 0
