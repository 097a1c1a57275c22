#!/bin/bash
# Round 3: PairHMM two problems per lane group (packed fp32, GASALX_HMM2=1 default) vs one
# (GASALX_HMM2=0): PairHMM parity tests under both, config 5 A/B, nvbio tests, kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l
mkdir -p $O
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "pairhmm or hmm" > $O/hmm2.txt 2>&1
rc=$?; echo "hmm tests (hmm2) rc=$rc"; tail -3 $O/hmm2.txt; if fatal $rc; then exit $rc; fi
GASALX_HMM2=0 timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread -k "pairhmm or hmm" > $O/hmm1.txt 2>&1
rc=$?; echo "hmm tests (hmm1) rc=$rc"; tail -3 $O/hmm1.txt; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_nvbio.py -x -q --timeout 300 --timeout-method thread > $O/nv.txt 2>&1
rc=$?; echo "nvbio tests rc=$rc"; tail -3 $O/nv.txt; if fatal $rc; then exit $rc; fi
for rep in 1 2; do
  for v in 1 0; do
    GASALX_HMM2=$v timeout -k 10 300 python -u bench.py --workload pairhmm --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 100000 > $O/hmm_v${v}_$rep.json 2> $O/hmm_v${v}_$rep.err
    rc=$?; echo "pairhmm hmm2=$v $rep rc=$rc $(python -c "import json;d=json.load(open('$O/hmm_v${v}_$rep.json'));print(d['value'],d['parity']['mismatches'],d['parity'].get('max_rel_err'))" 2>/dev/null)"
    if fatal $rc; then exit $rc; fi
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload pairhmm --steps 10 --warmup 2 --no-cpu --no-e2e --parity-pairs 0 > $GRAFT_REPO_ROOT/$O/prof.json 2>&1
echo "prof rc=$?"
exit 0
