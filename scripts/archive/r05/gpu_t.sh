#!/bin/bash
# round 5, session T: wave-synchronous 2 x 2 chunk reloads in tb_kernel's band walk.  GASAL
# traceback GPU tests, then config 3 one engine and three engines, then the one-engine kernel trace
# (the walk's time).  Output: gpurun_out/r05t/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/r05t; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "traceback or tb or config3 or cigar" > $O/tests.log 2>&1 || { tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
V=$ROOT/genomics-gpu_amd/lib/variants/libgasal_head.so   # HEAD (336eaad) built apart: the A side
for r in 1 2; do
  GASALX_LIB=$V timeout -k 10 300 python bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e > $O/head_s1_$r.json 2> $O/head_s1_$r.err || exit $?
  timeout -k 10 300 python bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e > $O/s1_$r.json 2> $O/s1_$r.err || exit $?
  GASALX_LIB=$V timeout -k 10 300 python bench.py --workload nw_tb --no-cpu --no-e2e > $O/head_s3_$r.json 2> $O/head_s3_$r.err || exit $?
  timeout -k 10 300 python bench.py --workload nw_tb --no-cpu --no-e2e > $O/s3_$r.json 2> $O/s3_$r.err || exit $?
  grep -o '"value": [0-9.]*' $O/head_s1_$r.json $O/s1_$r.json $O/head_s3_$r.json $O/s3_$r.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s1 -o run -- \
  python3 $ROOT/bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e --parity-pairs 1000 > $O/prof_s1.json 2> $O/prof_s1.err
echo "[prof] rc=$?"
