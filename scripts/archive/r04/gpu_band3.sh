#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04band3; mkdir -p $O
timeout -k 10 300 python -u tools/band_diag.py 8 64 600 > $O/diag1.log 2>&1; rc=$?; grep -v amdgpu.ids $O/diag1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_diag.py 20 310 700 > $O/diag2.log 2>&1; rc=$?; grep -v amdgpu.ids $O/diag2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "global or kat or config3 or traceback" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || { tail -30 $O/pytest.log; exit $rc; }
for v in "GASALX_TB_BAND=0" "GASALX_TB_BAND_W=12" "GASALX_TB_BAND_W=8" "GASALX_TB_BAND_W=16"; do
  env $v timeout -k 10 300 python bench.py --workload nw_tb --steps 10 --no-cpu --no-e2e --parity-pairs 100000 > "$O/nw_$v.json" 2> "$O/nw_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 "$O/nw_$v.err"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/nw_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'], d['parity']['by_field_rank0'], d['config']['plan'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_window_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/edges.log 2>&1
rc=$?; echo "edges rc=$rc $(tail -1 $O/edges.log)"; [ $rc -eq 0 ] || { tail -30 $O/edges.log; exit $rc; }
timeout -k 10 120 ./tools/ubench_issue > $O/ubench_issue.json 2> $O/ubench_issue.err; rc=$?; echo "ubench rc=$rc"; cat $O/ubench_issue.json
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "packed_input" > $O/packed.log 2>&1
rc=$?; echo "packed rc=$rc $(tail -1 $O/packed.log)"; [ $rc -eq 0 ] || { tail -30 $O/packed.log; exit $rc; }
timeout -k 10 300 python bench.py --workload semi --steps 10 --no-cpu --no-e2e --parity-pairs 200000 > $O/semi.json 2> $O/semi.err
rc=$?; echo "semi rc=$rc"; python -c "import json; d=json.loads(open('$O/semi.json').read().strip().splitlines()[-1]); print('semi', d['value'], d['ms_per_step'], d['parity']['mismatches'], d['config']['plan'])"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "with_start or start" > $O/start.log 2>&1
rc=$?; echo "start rc=$rc $(tail -1 $O/start.log)"; [ $rc -eq 0 ] || { tail -30 $O/start.log; exit $rc; }
for v in "GASALX_START_STOP=1" "GASALX_START_STOP=0"; do
  env $v timeout -k 10 300 python bench.py --workload sw_local_start --steps 10 --no-cpu --no-e2e --parity-pairs 200000 > "$O/st_$v.json" 2> "$O/st_$v.err"
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 "$O/st_$v.err"; exit $rc; }
  python -c "import json; d=json.loads(open('$O/st_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'], d['config']['plan'])"
done
timeout -k 10 300 python bench.py --workload sw_local --scores 2,4,6,1 --steps 10 --no-cpu --no-e2e --parity-pairs 200000 > $O/m2.json 2> $O/m2.err
rc=$?; echo "m2 rc=$rc"; python -c "import json; d=json.loads(open('$O/m2.json').read().strip().splitlines()[-1]); print('match2', d['value'], d['ms_per_step'], d['parity']['mismatches'], d['config']['plan'])"
