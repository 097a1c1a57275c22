#!/bin/bash
# Round 3 final pass, part C: the bench lines part B did not reach (KSW's pinned e2e
# timing lacked its seed scores, fixed in bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03fin2; mkdir -p $O
run() {  # run NAME ARGS...
  local n=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err
  local rc=$?; echo "$n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.loads(open('$O/bench_$n.json').read().strip().splitlines()[-1]); print('  ', d['value'], d['unit'], d['ms_per_step'], d.get('parity',{}).get('mismatches'), (d.get('roofline') or {}).get('traffic'))"
}
run ksw --workload ksw --steps 10 --no-cpu
run semi_banded --workload semi_banded --steps 10 --no-cpu
run nvbio_banded --workload nvbio_banded --steps 10 --no-cpu
