#!/bin/bash
# Round 3: SEMI drift frame (6 instructions per cell pair): semi GPU tests, then the
# config-4 bench lines and the semi path probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "semi or driver or multi" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for w in semi semi_start; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --no-cpu > $O/bench_$w.json 2> $O/bench_$w.err
  rc=$?; echo "$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python tools/path_probe.py 200000 semi_tt,semi_both,semi_query,semi_tt_start > $O/probe.jsonl 2> $O/probe.err
echo "probe rc=$?"
