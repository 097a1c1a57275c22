#!/bin/bash
# Round 3: SEMI tail offsets formed in the capture (fewer hoisted constants, fewer spills):
# semi GPU tests, config-4 bench and the TAIL=QUERY/BOTH probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03al; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "semi" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload semi --steps 10 --no-cpu --no-e2e > $O/bench_semi.json 2> $O/bench_semi.err
rc=$?; echo "semi rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.loads(open('$O/bench_semi.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatches'])"
timeout -k 10 300 python tools/path_probe.py 200000 semi_tt,semi_both,semi_query > $O/probe.jsonl 2> $O/probe.err
echo "probe rc=$?"; cat $O/probe.jsonl
