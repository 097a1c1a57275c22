#!/bin/bash
# round 4, session H: band pass fused into the checkpoint sweep (A/B against its own launch);
# PairHMM 4 waves default (A/B 3).  Output: gpurun_out/r04h/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04h; mkdir -p $O
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
run nw_tb "X=1" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_unfused "GASALX_LIB=genomics-gpu_amd/lib/variants/libgasal_unfused.so" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_w16 "GASALX_TB_BAND_W=16" nw_tb --steps 10 --parity-pairs 100000
run pairhmm "X=1" pairhmm --steps 10 --parity-pairs 100000
run pairhmm_3w "GASALX_LIB=genomics-gpu_amd/lib/variants/libgasal_hmm3.so" pairhmm --steps 10 --parity-pairs 100000
step hmmtests 300 $PYT tests/test_gpu_parity.py -k "pairhmm or hmm"
exit 0
