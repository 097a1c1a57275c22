#!/bin/bash
# Round 3: two engines on two streams, steps round-robin (test_prog.cpp NB_STREAMS = 2):
# does a step's traceback walk hide behind the next step's DP?  config 3, LOCAL+TB, and the
# score-only headline for neutrality; kernel trace of config 3 at two streams.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03v
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for wl in nw_tb sw_local_tb sw_local; do
  for rep in 1 2; do
    for st in 1 2; do
      timeout -k 10 300 python -u bench.py --workload $wl --streams $st --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/${wl}_s${st}_$rep.json 2> $O/${wl}_s${st}_$rep.err
      rc=$?; echo "$wl streams=$st rep=$rep rc=$rc $(python -c "import json;d=json.load(open('$O/${wl}_s${st}_$rep.json'));print(d['value'],d['ms_per_step'],d['parity']['mismatches'])" 2>/dev/null)"
      if fatal $rc; then exit $rc; fi
    done
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload nw_tb --streams 2 --steps 6 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > $GRAFT_REPO_ROOT/$O/prof.json 2>&1
echo "prof rc=$?"
exit 0
