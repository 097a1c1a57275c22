#!/bin/bash
# Round 3 final pass, part B: the whole GPU suite, smoke, and one bench line per
# workload at the final library (lines pick up profiles/pmc_<workload>.json).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03fin2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit $rc
run() {  # run NAME ARGS...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err
  local rc=$?; echo "$n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); print('  ', d['value'], d['unit'], d['ms_per_step'], d.get('parity',{}).get('mismatches'), (d.get('roofline') or {}).get('traffic'))"
}
run sw_local
run sw_local_start --workload sw_local_start --steps 10 --cpu-seconds 8
run sw_local_tb --workload sw_local_tb --steps 10 --no-cpu
run nw_tb --workload nw_tb --steps 10 --cpu-seconds 8
run semi --workload semi --steps 10 --cpu-seconds 8
run semi_start --workload semi_start --steps 10 --no-cpu
run pairhmm --workload pairhmm --steps 10 --cpu-seconds 8
run nvbio_gotoh --workload nvbio_gotoh --steps 10 --no-cpu
run ksw --workload ksw --steps 10 --no-cpu
run semi_banded --workload semi_banded --steps 10 --no-cpu
run nvbio_banded --workload nvbio_banded --steps 10 --no-cpu
