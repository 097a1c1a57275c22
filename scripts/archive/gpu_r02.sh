#!/bin/bash
# Round-2 GPU pass: parity tests, smoke, bench lines (each with its parity block),
# rocprof kernel-trace summaries.  Each GPU step has its own time limit; the script
# stops at the first step that faults, aborts or times out (124/134/137/139).
# Usage: gpu_r02.sh TAG [steps...]   steps: tests smoke bench prof (default: all)
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r02}; shift || true
WHAT=${*:-tests smoke bench prof}
O=gpurun_out/$TAG
mkdir -p "$O"
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 "$O/$name.out"
  if fatal $rc; then echo "fatal in $name"; tail -5 "$O/$name.err"; exit $rc; fi
  return 0
}
has() { [[ " $WHAT " == *" $1 "* ]]; }
if has tests; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
fi
if has smoke; then step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"; fi
if has bench; then
  step bench_sw_local 600 python bench.py
  step bench_cpu_plumbing 300 python bench.py --workload cpu_plumbing
  for w in ${BENCH_WORKLOADS:-nw_tb semi pairhmm sw_local_start sw_local_tb semi_start semi_banded}; do
    step bench_$w 600 python bench.py --workload $w --steps 10 --no-cpu
  done
fi
if has prof; then
  cd /tmp && export TMPDIR=/tmp
  for w in ${PROF_WORKLOADS:-sw_local nw_tb semi pairhmm}; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_$w" -o run -- python3 "$ROOT/bench.py" --workload $w --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > "$ROOT/$O/bench_prof_$w.out" 2> "$ROOT/$O/bench_prof_$w.err"
    rc=$?; echo "[rocprof $w] rc=$rc"
    if fatal $rc; then exit $rc; fi
  done
fi
exit 0
