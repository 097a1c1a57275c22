#!/bin/bash
# Round 3: traceback tail split (GASALX_TB_TAIL=1: whole DP rounds first, chunk 0's walk
# beside the tail's DP) vs one launch pair; parity tests under the split; kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03m
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
GASALX_TB_TAIL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_driver.py -x -q --timeout 300 --timeout-method thread -k "traceback or config3 or tb or cigar or driver" > $O/tb.txt 2>&1
rc=$?; echo "tb tests (tail split) rc=$rc"; tail -3 $O/tb.txt; if fatal $rc; then exit $rc; fi
for rep in 1 2; do
  for v in 1 0; do
    GASALX_TB_TAIL=$v timeout -k 10 300 python -u bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/nw_t${v}_$rep.json 2> $O/nw_t${v}_$rep.err
    rc=$?; echo "nw_tb tail=$v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/nw_t${v}_$rep.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
    if fatal $rc; then exit $rc; fi
  done
done
for v in 1 0; do
  GASALX_TB_TAIL=$v timeout -k 10 300 python -u bench.py --workload sw_local_tb --steps 5 --warmup 1 --no-cpu --no-e2e --parity-pairs 200000 > $O/swtb_t$v.json 2> $O/swtb_t$v.err
  rc=$?; echo "sw_local_tb tail=$v rc=$rc $(python -c "import json;d=json.load(open('$O/swtb_t$v.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
  if fatal $rc; then exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
GASALX_TB_TAIL=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload nw_tb --steps 3 --warmup 1 --no-cpu --no-e2e --parity-pairs 0 > $GRAFT_REPO_ROOT/$O/trace.json 2>&1
echo "trace rc=$?"
exit 0
