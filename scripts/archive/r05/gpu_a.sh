#!/bin/bash
# round 5, session A: GPU tests, the headline bench line, and config 5's three records of one
# library on one box (bench line, rocprofv3 kernel trace, PMC pass) -- VERDICT r04 item 1.
# Output: gpurun_out/r05a/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05a; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; fatal $rc && exit $rc
timeout -k 10 400 python bench.py > $O/bench_sw_local.json 2> $O/bench_sw_local.err
rc=$?; echo "sw_local rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_sw_local.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload pairhmm > $O/bench_pairhmm.json 2> $O/bench_pairhmm.err
rc=$?; echo "pairhmm rc=$rc $(grep -o '"value": [0-9.]*' $O/bench_pairhmm.json)"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pairhmm -o run -- \
  python3 $ROOT/bench.py --workload pairhmm --no-cpu --no-e2e > $O/prof_pairhmm.json 2> $O/prof_pairhmm.err
rc=$?; echo "prof pairhmm rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash $ROOT/scripts/pmc_session.sh r05a_pairhmm --workload pairhmm --parity-pairs 1000 || exit $?
exit 0
