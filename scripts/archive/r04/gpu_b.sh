#!/bin/bash
# round 4, session B: bench lines of the changed paths (A/B by environment), one box.
# Output: gpurun_out/r04b/<name>.json + a one-line summary per run on stdout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04b; mkdir -p $O
run() {  # name env workload [bench args...]
  local name=$1 envs=$2 w=$3; shift 3
  env $envs timeout -k 10 400 python bench.py --workload $w --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?
  [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -5 $O/$name.err; exit $rc; }
  python - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
p = d["parity"]
print(sys.argv[2], d["value"], "GCUPS", d["ms_per_step"], "ms", "kern", d["kernel_gcups"], "parity", p["pairs_checked"], p["mismatches"], d["config"]["plan"])
PY
}
run nw_tb "X=1" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_w8 "GASALX_TB_BAND_W=8" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_w16 "GASALX_TB_BAND_W=16" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_full "GASALX_TB_BAND=0" nw_tb --steps 10 --parity-pairs 100000
run sw_local "X=1" sw_local --steps 10 --parity-pairs 200000
run sw_local_300 "X=1" sw_local_300 --steps 5 --parity-pairs 100000
run m2_u16 "X=1" sw_local --scores 2,4,6,1 --steps 10 --parity-pairs 200000
run m2_seg "GASALX_KSEG=2" sw_local --scores 2,4,6,1 --steps 10 --parity-pairs 200000
run start_stop "X=1" sw_local_start --steps 5 --parity-pairs 200000
run start_nostop "GASALX_START_STOP=0" sw_local_start --steps 5 --parity-pairs 200000
run semi "X=1" semi --steps 5 --parity-pairs 200000
run pairhmm "X=1" pairhmm --steps 10 --parity-pairs 100000
exit 0
