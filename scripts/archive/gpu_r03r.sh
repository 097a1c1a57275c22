#!/bin/bash
# Round 3: ksw16 with the entry row in registers (QC 64/96/160; GASALX_KSW16_REG=0 = global
# array) vs the levels: KSW parity tests, probe at 200 K / 1 M, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03r
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "ksw" > $O/ksw.txt 2>&1
rc=$?; echo "ksw tests rc=$rc"; tail -2 $O/ksw.txt; if fatal $rc; then exit $rc; fi
for rep in 1 2; do
  for v in 1 0; do
    for np_ in 200000 1000000; do
      GASALX_KSW16_REG=$v timeout -k 10 300 python -u tools/path_probe.py $np_ ksw > $O/probe_r${v}_${np_}_$rep.jsonl 2> $O/probe_r${v}_${np_}_$rep.err
      rc=$?; echo "probe reg=$v pairs=$np_ $rep rc=$rc $(tail -1 $O/probe_r${v}_${np_}_$rep.jsonl)"
      if fatal $rc; then exit $rc; fi
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/path_probe.py 1000000 ksw > $GRAFT_REPO_ROOT/$O/prof.jsonl 2>&1
echo "prof rc=$?"
exit 0
