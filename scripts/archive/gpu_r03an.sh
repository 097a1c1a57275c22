#!/bin/bash
# Round 3: every planner path at the final library (tools/path_probe.py, 200 K pairs)
# and a second config-5 sample.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03an; mkdir -p $O
timeout -k 10 600 python tools/path_probe.py 200000 > $O/probe.jsonl 2> $O/probe.err
rc=$?; echo "probe rc=$rc"; cat $O/probe.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload pairhmm --steps 20 --no-cpu --no-e2e > $O/bench_pairhmm.json 2> $O/bench_pairhmm.err
rc=$?; echo "pairhmm rc=$rc"; python -c "import json; d=json.loads(open('$O/bench_pairhmm.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatches'])"
