#!/bin/bash
# round 4, session M: config 3 kernel breakdown on one stream (no overlap between the engines'
# kernels, so each launch's duration is its own), and the two-stream step beside it.
# Then the GLOBAL/TB parity tests and config 3 with the walk's lane regions staged in LDS
# (GASALX_TB_STAGE=1, default) and without.
# Output: gpurun_out/r04m/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O=$ROOT/gpurun_out/r04m; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- \
  python3 $ROOT/bench.py --no-cpu --no-e2e --workload nw_tb --streams 1 --steps 5 --warmup 1 --parity-pairs 1000 > $O/prof1.json 2> $O/prof1.err
rc=$?; echo "prof1 rc=$rc"; [ $rc -eq 0 ] || { tail -3 $O/prof1.err; exit $rc; }
python3 - $O/prof1/run_kernel_stats.csv <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 1), 'us', x['Percentage'][:5])
PY
cd $ROOT
timeout -k 10 300 python bench.py --workload nw_tb --no-cpu --no-e2e --streams 1 --steps 10 --parity-pairs 1000 > $O/s1.json 2> $O/s1.err
rc=$?; echo "s1 rc=$rc $(grep -o '"value": [0-9.]*' $O/s1.json)"
cd $ROOT
PYT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $PYT tests/test_gpu_parity.py -k "global or config3 or traceback" > $O/tbtests.log 2>&1
rc=$?; echo "tbtests rc=$rc $(tail -1 $O/tbtests.log)"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in 1 0; do
  GASALX_TB_STAGE=$v timeout -k 10 300 python bench.py --workload nw_tb --no-cpu --no-e2e --steps 10 --parity-pairs 100000 > $O/nw_tb_stage$v.json 2> $O/nw_tb_stage$v.err
  rc=$?; echo "nw_tb stage=$v rc=$rc $(grep -o '"value": [0-9.]*' $O/nw_tb_stage$v.json) $(grep -o '"mismatches": [0-9]*' $O/nw_tb_stage$v.json | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py --workload sw_local_tb --no-cpu --no-e2e --steps 5 --parity-pairs 100000 > $O/sw_local_tb.json 2> $O/sw_local_tb.err
rc=$?; echo "sw_local_tb rc=$rc $(grep -o '"value": [0-9.]*' $O/sw_local_tb.json) $(grep -o '"mismatches": [0-9]*' $O/sw_local_tb.json | head -1)"
exit 0
