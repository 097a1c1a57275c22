#!/bin/bash
# Round 3: packed SEMI TAIL=QUERY/BOTH/NONE parity + probe; nvbio reference vectors;
# int32-fallback probes of configs 2 and 4; headline line with the native CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03e
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "semiglobal" > $O/semi.txt 2>&1
rc=$?; echo "semi rc=$rc"; tail -3 $O/semi.txt; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_nvbio.py -x -q --timeout 200 --timeout-method thread -k reference > $O/nv.txt 2>&1
rc=$?; echo "nv rc=$rc"; tail -2 $O/nv.txt; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u tools/path_probe.py 200000 semi_tt,semi_both,semi_query,semi_none > $O/probe.jsonl 2> $O/probe.err
rc=$?; echo "probe rc=$rc"; cat $O/probe.jsonl; if fatal $rc; then exit $rc; fi
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err; rc=$?
  echo "$n rc=$rc $(python -c "import json;d=json.load(open('$O/$n.json'));print(d['value'],d['config']['plan'],d['parity']['mismatches'],d.get('cpu_baseline',{}).get('value'),d.get('cpu_baseline',{}).get('build'))" 2>/dev/null)"; return $rc; }
run sw_local_i32 --workload sw_local --force-int32 --steps 10 --warmup 2 --no-cpu --no-e2e || { fatal $? && exit 1; }
run sw_local_m2 --workload sw_local --scores 2,4,6,1 --steps 10 --warmup 2 --no-cpu --no-e2e || { fatal $? && exit 1; }
run semi_i32 --workload semi --force-int32 --steps 5 --warmup 1 --no-cpu --no-e2e --parity-pairs 1000000 || { fatal $? && exit 1; }
run sw_local --workload sw_local --steps 20 --warmup 3 || { fatal $? && exit 1; }
exit 0
