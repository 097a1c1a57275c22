#!/bin/bash
# Band-recomputation traceback: GLOBAL TB parity tests, then config 3 A/B (band vs full matrix, w).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04band1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "global or kat or config3 or traceback" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit $rc; }
for v in "GASALX_TB_BAND=0" "GASALX_TB_BAND_W=12" "GASALX_TB_BAND_W=8" "GASALX_TB_BAND_W=16"; do
  env $v timeout -k 10 300 python bench.py --workload nw_tb --steps 10 --no-cpu --no-e2e --parity-pairs 100000 > "$O/nw_$v.json" 2> "$O/nw_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 "$O/nw_$v.err"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/nw_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'], d['config']['plan'])"
done
