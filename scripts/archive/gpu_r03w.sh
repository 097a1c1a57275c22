#!/bin/bash
# Round 3: bench default of two engines on two streams: multi-rank (gloo, one GPU) path,
# config 3 and the headline at the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03w
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py > $O/multi.log 2>&1
rc=$?; echo "multi rc=$rc $(tail -1 $O/multi.log)"; if [ $rc -ne 0 ]; then exit $rc; fi
for wl in nw_tb sw_local; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/${wl}.json 2> $O/${wl}.err
  rc=$?; echo "$wl rc=$rc $(python -c "import json;d=json.load(open('$O/${wl}.json'));print(d['value'],d['ms_per_step'],d['parity']['mismatches'],d['config'].get('streams'))" 2>/dev/null)"
  if fatal $rc; then exit $rc; fi
done
exit 0
