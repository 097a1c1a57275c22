#!/bin/bash
# Round 3: ksw16 occupancy A/B (8 waves/SIMD default vs 7, variant kw7) at 200 K / 1 M pairs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03o
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "ksw" > $O/ksw.txt 2>&1
rc=$?; echo "ksw tests rc=$rc"; tail -2 $O/ksw.txt; if fatal $rc; then exit $rc; fi
for rep in 1 2; do
  for v in base kw7; do
    if [ $v = base ]; then L=""; else L="$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"; fi
    for np_ in 200000 1000000; do
      GASALX_LIB=$L timeout -k 10 300 python -u tools/path_probe.py $np_ ksw > $O/probe_${v}_${np_}_$rep.jsonl 2> $O/probe_${v}_${np_}_$rep.err
      rc=$?; echo "probe $v pairs=$np_ $rep rc=$rc $(tail -1 $O/probe_${v}_${np_}_$rep.jsonl)"
      if fatal $rc; then exit $rc; fi
    done
  done
done
exit 0
