#!/bin/bash
# traceback tests, then the two traceback workloads under rocprofv3 (walk kernel time)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out/${1:-s5}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "traceback or tb or pipeline or driver" > "$O/t.out" 2>&1
rc=$?
tail -2 "$O/t.out"; grep -E "^E " "$O/t.out" | head -5
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for w in nw_tb sw_local_tb; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_$w" -o run -- python3 "$ROOT/bench.py" --workload $w --steps 10 --warmup 2 --no-cpu --no-e2e > "$ROOT/$O/b_$w.json" 2> "$ROOT/$O/b_$w.err" || exit $?
  echo "$w $(cut -c100-200 "$ROOT/$O/b_$w.json")"
  grep -E "tb_kernel|wf16" "$ROOT/$O/prof_$w/run_kernel_stats.csv" | cut -d, -f1-4
done
exit 0
