#!/bin/bash
# round 4, session G: band pass with the per-lane stream blocks; GLOBAL score sweep; phase A at
# 2 waves (variant).  Output: gpurun_out/r04g/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r04g; mkdir -p $O
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
run nw_tb "X=1" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_w16 "GASALX_TB_BAND_W=16" nw_tb --steps 10 --parity-pairs 100000
run nw_tb_cp2 "GASALX_LIB=genomics-gpu_amd/lib/variants/libgasal_cp2.so" nw_tb --steps 10 --parity-pairs 100000
run nw_score "X=1" nw_score --steps 10 --parity-pairs 100000
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nw_tb -o run -- \
  python3 $ROOT/bench.py --no-cpu --no-e2e --workload nw_tb --steps 5 --warmup 1 --streams 1 --parity-pairs 20000 > $O/prof_nw_tb.json 2> $O/prof_nw_tb.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/prof_nw_tb -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("   %-70s calls %5s avg %10.1f us" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
exit 0
