#!/bin/bash
# the bench line of every workload with its CPU baseline, end-to-end
# columns and parity (bench.py picks up profiles/pmc_<w>.json of the same library and plan).
# Output: gpurun_out/$REPRO_TAG (default repro)/bench_<w>.json
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/${REPRO_TAG:-repro}; mkdir -p $O
for w in ${WORKLOADS:-sw_local nw_tb semi pairhmm sw_local_300 sw_local_start sw_local_tb semi_start semi_banded nvbio_gotoh nvbio_banded ksw nw_score cpu_plumbing}; do
  timeout -k 10 400 python3 bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err
  rc=$?
  python3 - "$O/bench_$w.json" "$w" "$rc" <<'PY'
import json, sys
try:
    d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
    p = d.get("parity") or {}
    print(sys.argv[2], "rc", sys.argv[3], d["value"], d["unit"], "parity", p.get("pairs_checked"), p.get("mismatches"),
          "cpu", (d.get("cpu_baseline") or {}).get("value"), flush=True)
except Exception as e:
    print(sys.argv[2], "rc", sys.argv[3], "no line", e, flush=True)
PY
  case $rc in 0) ;; *) tail -3 $O/bench_$w.err; exit $rc;; esac
done
exit 0
