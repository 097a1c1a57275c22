#!/bin/bash
# round 6 baseline on a fresh box: config 2 and config 3 lines (one engine and three), plus a
# kernel trace of config 3 on one stream (where a call's time goes).  Output: gpurun_out/r06base/
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd $ROOT
O=$ROOT/gpurun_out/${TAG:-r06base}; mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.json" 2> "$O/$name.err"
  local rc=$?
  echo "[$name] rc=$rc $(grep -o '"value": [0-9.]*' $O/$name.json | head -1)"
  if fatal $rc; then echo "fatal in $name"; exit $rc; fi
  return 0
}
step bench_default 300 python bench.py --no-cpu --no-e2e
step bench_nw_tb 300 python bench.py --workload nw_tb --no-cpu --no-e2e
step bench_nw_tb_s1 300 python bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nw_tb_s1 -o run -- \
  python3 $ROOT/bench.py --workload nw_tb --streams 1 --no-cpu --no-e2e --parity-pairs 1000 --steps 10 > $O/prof_nw_tb_s1.json 2> $O/prof_nw_tb_s1.err
rc=$?; echo "[prof nw_tb s1] rc=$rc"
exit 0
