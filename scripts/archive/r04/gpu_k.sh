#!/bin/bash
# round 4, session K: diagonal-major band flags; band width sweep; reverse-pass prep split; config-3 counters.
# Output: gpurun_out/r04k/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04k; mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc $(tail -1 $O/$name.log)"
  [ $rc -eq 0 ] || grep -E "^FAILED|^ERROR" $O/$name.log | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
run() {
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
PYT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread"
step tbtests 600 $PYT tests/test_gpu_parity.py -k "global or config3 or traceback"
step edges 300 $PYT tests/test_gpu_window_edges.py -k "global"
for w in 8 10 12 16; do run nw_tb_w$w "GASALX_TB_BAND_W=$w" nw_tb --steps 10 --parity-pairs 100000; done
step starttests 600 $PYT tests/test_gpu_parity.py -k "start"
run start "X=1" sw_local_start --steps 5 --parity-pairs 200000
run semi_start "X=1" semi_start --steps 3 --parity-pairs 200000
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- \
    python3 $ROOT/bench.py --no-cpu --no-e2e --steps 2 --warmup 1 --workload nw_tb --streams 1 --parity-pairs 1000 > $O/pmc_$c.json 2> $O/pmc_$c.err
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
