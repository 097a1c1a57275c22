#!/bin/bash
# PairHMM pass: parity tests, config-5 bench line, rocprof kernel-trace summary.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
O=gpurun_out/${1:-hmm}; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "pairhmm or hmm" > "$O/pytest.out" 2>&1 || { tail -30 "$O/pytest.out"; exit 1; }
tail -2 "$O/pytest.out"
timeout -k 10 400 python bench.py --workload pairhmm --steps 10 > "$O/bench.json" 2> "$O/bench.err" || exit $?
tail -c 600 "$O/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$O/prof" -o run -- python3 "$ROOT/bench.py" --workload pairhmm --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > "$ROOT/$O/prof.out" 2> "$ROOT/$O/prof.err"
echo "rocprof rc=$?"
