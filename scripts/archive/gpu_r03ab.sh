#!/bin/bash
# Round 3: GLOBAL drift e (7 instructions per cell pair): global GPU tests, config-3
# bench line, global path probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "global or driver or multi or nw or config3 or traceback" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload nw_tb --steps 10 --no-cpu > $O/bench_nw_tb.json 2> $O/bench_nw_tb.err
rc=$?; echo "nw_tb rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/path_probe.py 200000 global,global_tb > $O/probe.jsonl 2> $O/probe.err
echo "probe rc=$?"
