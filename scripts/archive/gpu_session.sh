#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first GPU step that faults, aborts or times out (exit 124/134/137/139).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01}
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }

timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu_${TAG}.log
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_${TAG}.log
if fatal $rc; then exit $rc; fi

timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_${TAG}.json; tail -3 gpurun_out/bench_${TAG}.err
if fatal $rc; then exit $rc; fi

cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}" -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/bench_prof_${TAG}.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG}.err"
rc=$?; echo "rocprof rc=$rc"
exit 0
