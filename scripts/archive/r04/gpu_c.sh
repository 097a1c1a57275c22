#!/bin/bash
# round 4, session C: micro-benchmark, the changed paths' parity tests, then bench lines
# (A/B by environment / variant library).  Output: gpurun_out/r04c/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04c; mkdir -p $O
step() {  # name timeout cmd...: run, report, stop the session on failure
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log)"
  [ $rc -eq 0 ] || { tail -40 $O/$name.log; exit $rc; }
}
run() {  # name env workload [bench args...]
  local name=$1 envs=$2 w=$3; shift 3
  env $envs timeout -k 10 300 python bench.py --workload $w --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $O/$name.err; exit $rc; }
  python - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
p = d["parity"]
print(sys.argv[2], d["value"], "GCUPS", d["ms_per_step"], "ms kern", d["kernel_gcups"], "parity", p["pairs_checked"], p["mismatches"], d["config"]["plan"], flush=True)
PY
}
PYT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread"
step ubench 120 ./tools/ubench_issue
run sw_local "X=1" sw_local --steps 10 --parity-pairs 200000
run sw_local_ukey0 "GASALX_LIB=genomics-gpu_amd/lib/variants/libgasal_ukey0.so" sw_local --steps 10 --parity-pairs 200000
step localtests 600 $PYT tests/test_gpu_parity.py -k "local"
step tbtests 600 $PYT tests/test_gpu_parity.py -k "global or kat or config3 or traceback"
run nw_tb "X=1" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_full "GASALX_TB_BAND=0" nw_tb --steps 10 --parity-pairs 100000
run sw_local_tb "X=1" sw_local_tb --steps 6 --parity-pairs 100000
run sw_local_tb_old "GASALX_LTBD=0" sw_local_tb --steps 6 --parity-pairs 100000
run sw_local_300 "X=1" sw_local_300 --steps 5 --parity-pairs 50000
run semi "X=1" semi --steps 5 --parity-pairs 200000
run pairhmm "X=1" pairhmm --steps 10 --parity-pairs 100000
run start_stop "X=1" sw_local_start --steps 5 --parity-pairs 200000
step edges 600 $PYT tests/test_gpu_window_edges.py
exit 0
