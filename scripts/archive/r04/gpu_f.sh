#!/bin/bash
# round 4, session F: rocprofv3 kernel-trace summaries (config 3 band traceback, one stream and
# two; PairHMM 3 and 4 waves).  Output: gpurun_out/r04f/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/r04f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
prof() {  # name env bench-args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- \
    python3 $ROOT/bench.py --no-cpu --no-e2e "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $O/$name.err; exit $rc; }
  f=$(find $O/$name -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("   %-70s calls %5s avg %10.1f us total %8.2f ms" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
}
prof nw_tb_s1 "X=1" --workload nw_tb --steps 5 --warmup 1 --streams 1 --parity-pairs 20000
prof nw_tb_s1_w8 "GASALX_TB_BAND_W=8" --workload nw_tb --steps 5 --warmup 1 --streams 1 --parity-pairs 20000
prof nw_tb_s1_full "GASALX_TB_BAND=0" --workload nw_tb --steps 5 --warmup 1 --streams 1 --parity-pairs 20000
prof pairhmm_3w "X=1" --workload pairhmm --steps 5 --warmup 1 --parity-pairs 20000
prof pairhmm_4w "GASALX_LIB=$ROOT/genomics-gpu_amd/lib/variants/libgasal_hmm4.so" --workload pairhmm --steps 5 --warmup 1 --parity-pairs 20000
exit 0
