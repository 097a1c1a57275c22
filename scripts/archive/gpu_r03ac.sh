#!/bin/bash
# Round 3: LOCAL f16-pattern paired keys (10.5 instructions per cell pair): local GPU
# tests, headline bench (A/B against GASALX_KF16=0), local probes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03ac}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "local or driver or config2 or sample or smoke or kat or reference or multi or start" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench_sw_local.json 2> $O/bench_sw_local.err
rc=$?; echo "sw_local rc=$rc"; [ $rc -eq 0 ] || exit $rc
GASALX_KF16=0 timeout -k 10 300 python bench.py --steps 20 --no-cpu > $O/bench_sw_local_kf0.json 2> $O/bench_sw_local_kf0.err
rc=$?; echo "sw_local kf0 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload sw_local_start --steps 10 --no-cpu > $O/bench_sw_local_start.json 2> $O/bench_sw_local_start.err
rc=$?; echo "sw_local_start rc=$rc"; [ $rc -eq 0 ] || exit $rc
