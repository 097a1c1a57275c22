#!/bin/bash
# round 4, session U: PairHMM's last round on twice the lanes (GASALX_HMM_TAIL, default on) against
# one launch; the PairHMM GPU tests.
# Output: gpurun_out/r04u/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/ -m gpu -q -k hmm --timeout 120 --timeout-method thread > $O/hmm_tests.log 2>&1
rc=$?; echo "hmm tests rc=$rc $(tail -1 $O/hmm_tests.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for t in 1 0 1 0; do
  GASALX_HMM_TAIL=$t timeout -k 10 300 python bench.py --workload pairhmm --no-cpu --no-e2e --steps 10 --parity-pairs 100000 > $O/hmm_tail$t.json 2> $O/hmm_tail$t.err
  rc=$?; echo "tail=$t rc=$rc $(grep -o '"value": [0-9.]*' $O/hmm_tail$t.json) $(grep -o '"mismatches": [0-9]*' $O/hmm_tail$t.json | head -1)"
  [ $rc -eq 0 ] || { tail -5 $O/hmm_tail$t.err; exit $rc; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python3 $ROOT/bench.py --no-cpu --no-e2e --workload pairhmm --steps 5 --warmup 1 --parity-pairs 1000 > $O/prof.json 2> $O/prof.err
echo "prof rc=$?"
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 1), 'us')
PY
