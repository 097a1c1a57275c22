#!/bin/bash
# A/B the GLOBAL+TB build variants (lib/variants): TB parity subset + nw_tb bench each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/tune_tb
O=gpurun_out/tune_tb
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for so in default genomics-gpu_amd/lib/variants/libgasal_*.so; do
  if [ "$so" = default ]; then n=default; unset GASALX_LIB; else n=$(basename "$so" .so); n=${n#libgasal_}; export GASALX_LIB=$PWD/$so; fi
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "global or traceback or packed" > $O/pytest_$n.log 2>&1
  rc=$?; echo "$n pytest rc=$rc $(tail -1 $O/pytest_$n.log)"
  if fatal $rc; then exit $rc; fi
  timeout -k 10 300 python bench.py --workload nw_tb --steps 10 --warmup 2 --no-cpu > $O/bench_$n.json 2> $O/bench_$n.err
  rc=$?; echo "$n bench rc=$rc"; python -c "import json;d=json.load(open('$O/bench_$n.json'));print(d['value'],d.get('kernel_gcups'))" || true
  if fatal $rc; then exit $rc; fi
done
exit 0
