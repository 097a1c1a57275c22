#!/bin/bash
# Round 3: traceback flags as one v_pk_sub_u16 each (default) vs the round-2 biased
# 32-bit form (variant fadd): parity + config 3 + LOCAL+TB A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03i
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_driver.py -x -q --timeout 300 --timeout-method thread -k "traceback or config3 or tb or cigar or driver" > $O/tb.txt 2>&1
rc=$?; echo "tb rc=$rc"; tail -3 $O/tb.txt; if fatal $rc; then exit $rc; fi
for rep in 1 2; do
  for v in base fadd; do
    if [ $v = base ]; then L=""; else L="$PWD/genomics-gpu_amd/lib/variants/libgasal_$v.so"; fi
    GASALX_LIB=$L timeout -k 10 300 python -u bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/nw_${v}_$rep.json 2> $O/nw_${v}_$rep.err
    rc=$?; echo "nw_tb $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/nw_${v}_$rep.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
    if fatal $rc; then exit $rc; fi
    GASALX_LIB=$L timeout -k 10 300 python -u bench.py --workload sw_local_tb --steps 5 --warmup 1 --no-cpu --no-e2e --parity-pairs 200000 > $O/swtb_${v}_$rep.json 2> $O/swtb_${v}_$rep.err
    rc=$?; echo "sw_local_tb $v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/swtb_${v}_$rep.json'));print(d['value'],d['parity']['mismatches'])" 2>/dev/null)"
    if fatal $rc; then exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_nw -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > $GRAFT_REPO_ROOT/$O/prof_nw.json 2>&1
echo "prof rc=$?"
exit 0
