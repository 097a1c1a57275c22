#!/bin/bash
# Focused GPU pass: a pytest -k selection (arg 2) with its own time limit; logs under gpurun_out/TAG.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-quick}; SEL=${2:-}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  ${SEL:+-k "$SEL"} > "$O/pytest.out" 2> "$O/pytest.err"
rc=$?
tail -25 "$O/pytest.out"
exit $rc
