#!/bin/bash
# Round 3: SEMI TAIL=QUERY/BOTH waves A/B (R = 23: 2 waves vs 3 with spills) + kernel split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03f
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for rep in 1 2; do
  for v in base tq3; do
    if [ $v = base ]; then L=""; else L="$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"; fi
    GASALX_LIB=$L timeout -k 10 300 python -u tools/path_probe.py 200000 semi_tt,semi_both,semi_query > $O/probe_${v}_$rep.jsonl 2> $O/probe_${v}_$rep.err
    rc=$?; echo "$v $rep rc=$rc"; cat $O/probe_${v}_$rep.jsonl; if fatal $rc; then exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/path_probe.py 200000 semi_both > $GRAFT_REPO_ROOT/$O/prof.txt 2>&1
echo "prof rc=$?"
exit 0
