#!/bin/bash
# Round 3: interleaved direction chunks (8 consecutive pairs, default) vs per-pair
# (GASALX_TB_Q8=0): traceback parity + config 3 + LOCAL+TB A/B, then chunk pipeline sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03j
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_driver.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread -k "traceback or config3 or tb or cigar or driver" > $O/tb.txt 2>&1
rc=$?; echo "tb rc=$rc"; tail -3 $O/tb.txt; if fatal $rc; then exit $rc; fi
for rep in 1 2; do
  for v in 1 0; do
    GASALX_TB_Q8=$v timeout -k 10 300 python -u bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/nw_q${v}_$rep.json 2> $O/nw_q${v}_$rep.err
    rc=$?; echo "nw_tb q8=$v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/nw_q${v}_$rep.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
    if fatal $rc; then exit $rc; fi
    GASALX_TB_Q8=$v timeout -k 10 300 python -u bench.py --workload sw_local_tb --steps 5 --warmup 1 --no-cpu --no-e2e --parity-pairs 200000 > $O/swtb_q${v}_$rep.json 2> $O/swtb_q${v}_$rep.err
    rc=$?; echo "sw_local_tb q8=$v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/swtb_q${v}_$rep.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
    if fatal $rc; then exit $rc; fi
  done
done
for ch in 2 3; do
  GASALX_TB_CHUNKS=$ch timeout -k 10 300 python -u bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/nw_ch$ch.json 2> $O/nw_ch$ch.err
  rc=$?; echo "nw_tb chunks=$ch rc=$rc $(python -c "import json;d=json.load(open('$O/nw_ch$ch.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
  if fatal $rc; then exit $rc; fi
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_nw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > $GRAFT_REPO_ROOT/$O/prof_nw.json 2>&1
echo "prof rc=$?"
exit 0
