#!/bin/bash
# rocprofv3 kernel-trace summaries of every bench workload, then the PMC
# passes (scripts/pmc_session.sh: separate --pmc runs, never with traces) of the main ones.
# Output: gpurun_out/$REPRO_TAG (default repro)/prof_<w>/, gpurun_out/pmc_<w>/ (summarise with tools/pmc_summary.py)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$ROOT/gpurun_out/${REPRO_TAG:-repro}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in sw_local nw_tb semi pairhmm sw_local_300 sw_local_start sw_local_tb semi_start semi_banded nvbio_gotoh nvbio_banded ksw nw_score; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- \
    python3 $ROOT/bench.py --no-cpu --no-e2e --workload $w --steps 5 --warmup 1 --parity-pairs 20000 > $O/prof_$w.json 2> $O/prof_$w.err
  rc=$?; echo "prof $w rc=$rc"
  case $rc in 0) ;; *) tail -3 $O/prof_$w.err; exit $rc;; esac
done
for w in sw_local semi nw_tb pairhmm sw_local_300; do
  bash $ROOT/scripts/pmc_session.sh $w --workload $w --parity-pairs 1000 || exit $?
done
exit 0
