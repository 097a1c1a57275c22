#!/bin/bash
# Round 3: KSW two pairs per lane (ksw16.hpp, default) vs the thread-per-pair levels
# (GASALX_KSW16=0): KSW parity tests, path probe at 200 K and 1 M pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03n
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "ksw" > $O/ksw.txt 2>&1
rc=$?; echo "ksw tests rc=$rc"; tail -3 $O/ksw.txt; if fatal $rc; then exit $rc; fi
for v in 1 0; do
  for np_ in 200000 1000000; do
    GASALX_KSW16=$v timeout -k 10 300 python -u tools/path_probe.py $np_ ksw > $O/probe_k${v}_$np_.jsonl 2> $O/probe_k${v}_$np_.err
    rc=$?; echo "probe ksw16=$v pairs=$np_ rc=$rc $(cat $O/probe_k${v}_$np_.jsonl | tail -1)"
    if fatal $rc; then exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/path_probe.py 1000000 ksw > $GRAFT_REPO_ROOT/$O/prof.jsonl 2>&1
echo "prof rc=$?"
exit 0
