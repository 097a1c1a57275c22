set -u
mkdir -p gpurun_out/k2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "local or sample or start or driver" > gpurun_out/k2/t.out 2>&1
rc=$?; tail -2 gpurun_out/k2/t.out; grep -E "^E " gpurun_out/k2/t.out | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/sample_probe.py 1000000 > gpurun_out/k2/p1m.out 2>&1 || exit $?
cat gpurun_out/k2/p1m.out | grep mode
GASALX_LIB=$PWD/genomics-gpu_amd/lib/variants/libgasal_k2w3.so timeout -k 10 300 python tools/sample_probe.py 1000000 local > gpurun_out/k2/p1m_w3.out 2>&1 || exit $?
grep mode gpurun_out/k2/p1m_w3.out
timeout -k 10 300 python tools/sample_probe.py 5000 local,semi_tt > gpurun_out/k2/p5k.out 2>&1 || exit $?
grep mode gpurun_out/k2/p5k.out
