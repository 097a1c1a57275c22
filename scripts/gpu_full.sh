#!/bin/bash
# The whole GPU suite (one process) + smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-full}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/tests.txt
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.txt
exit $rc
