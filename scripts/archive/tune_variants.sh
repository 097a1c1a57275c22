#!/bin/bash
# A/B the packed-kernel build variants in lib/variants: LOCAL parity subset + short bench each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
for so in genomics-gpu_amd/lib/variants/libgasal_*.so; do
  n=$(basename "$so" .so); n=${n#libgasal_}
  export GASALX_LIB=$PWD/$so
  timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "local or packed" > gpurun_out/tune_pytest_$n.log 2>&1
  rc=$?; echo "$n pytest rc=$rc $(tail -1 gpurun_out/tune_pytest_$n.log)"
  if fatal $rc; then exit $rc; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/tune_bench_$n.json 2> gpurun_out/tune_bench_$n.err
  rc=$?; echo "$n bench rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/tune_bench_$n.json'));print(d['value'],d.get('kernel_gcups'),d['roofline'].get('achieved'))" || true
  if fatal $rc; then exit $rc; fi
done
exit 0
