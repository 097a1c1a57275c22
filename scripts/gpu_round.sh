#!/bin/bash
# Full GPU pass: parity tests, smoke, bench lines for every workload, rocprof kernel
# trace of the headline bench.  Every GPU step has its own time limit; the script
# stops at the first step that faults, aborts or times out (124/134/137/139).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r01}
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
step pytest_gpu 1200 python -m pytest tests -m gpu -q -x
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench_sw_local 600 python bench.py
step bench_nw_tb 600 python bench.py --workload nw_tb --no-cpu --steps 10
step bench_semi 600 python bench.py --workload semi --no-cpu --steps 10
step bench_pairhmm 600 python bench.py --workload pairhmm --steps 10 --cpu-seconds 8
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_sw_local" -o run -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$ROOT/$O/bench_prof.out" 2> "$ROOT/$O/bench_prof.err"
echo "[rocprof] rc=$?"
exit 0
