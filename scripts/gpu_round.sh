#!/bin/bash
# Full GPU pass: parity tests, smoke, bench lines for every workload, rocprof kernel
# trace (kernel-only runs: --no-e2e, so the per-kernel averages are the timed launches)
# of every workload.  Every GPU step has its own time limit; the script stops at the
# first step that faults, aborts or times out (124/134/137/139).
# Usage: gpu_round.sh TAG [pytest -k expression]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r01}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 "$O/$name.out"
  if fatal $rc; then echo "fatal in $name"; exit $rc; fi
  return 0
}
if [ -n "$K" ]; then
  step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K"
else
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_sw_local 600 python bench.py
step bench_sw_local_start 600 python bench.py --workload sw_local_start --steps 10 --cpu-seconds 8
step bench_nw_tb 600 python bench.py --workload nw_tb --no-cpu --steps 10
step bench_sw_local_tb 600 python bench.py --workload sw_local_tb --no-cpu --steps 10
step bench_semi 600 python bench.py --workload semi --no-cpu --steps 10
step bench_semi_start 600 python bench.py --workload semi_start --no-cpu --steps 10
step path_probe 600 python tools/path_probe.py 200000
step bench_pairhmm 600 python bench.py --workload pairhmm --steps 10 --cpu-seconds 8
cd /tmp && export TMPDIR=/tmp
for w in ${PROF_WORKLOADS:-sw_local sw_local_start sw_local_tb nw_tb semi semi_start pairhmm}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_$w" -o run -- python3 "$ROOT/bench.py" --workload $w --steps 10 --warmup 2 --no-cpu --no-e2e > "$ROOT/$O/bench_prof_$w.out" 2> "$ROOT/$O/bench_prof_$w.err"
  rc=$?; echo "[rocprof $w] rc=$rc"
  if fatal $rc; then exit $rc; fi
done
exit 0
