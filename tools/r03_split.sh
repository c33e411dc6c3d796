# split-bf16 fp32 GEMM: accuracy tests + per-shape timing against the native f32 / bf16 kernels; fused a2f core
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROWS=8192 PREC=fp32,fp32s,fp32s2,bf16 timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/r03_gemm_split.log 2>&1 || { cat gpurun_out/r03_gemm_split.log | tail -20; exit 5; }
cat gpurun_out/r03_gemm_split.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_x2y.py tests/test_gpu_split.py tests/test_gpu_parity.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_split_test.log 2>&1
rc=$?; grep -E "PASS|FAIL|max \|err|^E " gpurun_out/r03_split_test.log | head -60; exit $rc
