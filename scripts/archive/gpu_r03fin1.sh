#!/bin/bash
# Round 3 final pass, part 1: the whole GPU suite, smoke, and the GLOBAL+TB 3-wave A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03fin1; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $O/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; [ $rc -eq 0 ] || exit $rc
for v in base tb3 tb3i; do
  lib=""; [ "$v" != base ] && lib="GASALX_LIB=$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"
  env $lib timeout -k 10 300 python bench.py --workload nw_tb --steps 10 --no-cpu --no-e2e --parity-pairs 20000 > "$O/tb_$v.json" 2> "$O/tb_$v.err"
  rc=$?; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.loads(open('$O/tb_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity']['mismatches'])"
done
timeout -k 10 300 python bench.py --workload pairhmm --steps 10 --no-cpu > $O/bench_pairhmm.json 2> $O/bench_pairhmm.err
rc=$?; echo "pairhmm rc=$rc"; python -c "import json; d=json.loads(open('$O/bench_pairhmm.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity'])"
timeout -k 10 300 python bench.py --workload sw_local_tb --steps 10 --no-cpu > $O/bench_sw_local_tb.json 2> $O/bench_sw_local_tb.err
rc=$?; echo "sw_local_tb rc=$rc"; python -c "import json; d=json.loads(open('$O/bench_sw_local_tb.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatches'], d['config'].get('plan'))"
GASALX_KF16=0 timeout -k 10 300 python bench.py --workload sw_local_tb --steps 10 --no-cpu > $O/bench_sw_local_tb_kf0.json 2> $O/bench_sw_local_tb_kf0.err
rc=$?; echo "sw_local_tb kf0 rc=$rc"; python -c "import json; d=json.loads(open('$O/bench_sw_local_tb_kf0.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['mismatches'])"
