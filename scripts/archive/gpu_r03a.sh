#!/bin/bash
# Round 3: multi-GPU tests, traceback parity, config-3 chunk sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
O=gpurun_out/r03a
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 300 --timeout-method thread > $O/multi.txt 2>&1
rc=$?; echo "multi rc=$rc"; tail -3 $O/multi.txt; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "traceback or config3 or tb or gainful" > $O/tb.txt 2>&1
rc=$?; echo "tb rc=$rc"; tail -3 $O/tb.txt; if fatal $rc; then exit $rc; fi
for c in 1 2 4 8; do
  GASALX_TB_CHUNKS=$c timeout -k 10 300 python -u bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/nw_tb_c$c.json 2> $O/nw_tb_c$c.err
  rc=$?; echo "nw_tb chunks=$c rc=$rc $(python -c "import json;d=json.load(open('$O/nw_tb_c$c.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
  if fatal $rc; then exit $rc; fi
done
for c in 1 4; do
  GASALX_TB_CHUNKS=$c timeout -k 10 300 python -u bench.py --workload sw_local_tb --steps 5 --warmup 1 --no-cpu --no-e2e --parity-pairs 200000 > $O/swtb_c$c.json 2> $O/swtb_c$c.err
  rc=$?; echo "sw_local_tb chunks=$c rc=$rc $(python -c "import json;d=json.load(open('$O/swtb_c$c.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
  if fatal $rc; then exit $rc; fi
done
exit 0
