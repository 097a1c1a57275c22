#!/bin/bash
# Round 3 final pass, part A: rocprofv3 kernel-trace summaries (--no-e2e: the per-kernel
# averages are the timed launches) and the PMC passes (scripts/pmc_session.sh) of the
# bench workloads, at the final library.  Every GPU step under its own time limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out/r03fin3; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
cd /tmp && export TMPDIR=/tmp
for w in sw_local nw_tb semi pairhmm nvbio_gotoh sw_local_start sw_local_tb semi_start; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof_$w" -o run -- python3 "$ROOT/bench.py" --workload $w --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > "$ROOT/$O/bench_prof_$w.out" 2> "$ROOT/$O/bench_prof_$w.err"
  rc=$?; echo "[rocprof $w] rc=$rc"
  if fatal $rc; then exit $rc; fi
done
cd "$ROOT"
bash scripts/pmc_r03.sh sw_local nw_tb semi pairhmm nvbio_gotoh sw_local_start sw_local_tb semi_start
