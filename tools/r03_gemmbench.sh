set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROWS=8192 PREC=${PRECS:-fp32,fp32s,bf16} timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/r03_gemm_bench2.log 2>&1 || { tail -20 gpurun_out/r03_gemm_bench2.log; exit 5; }
cat gpurun_out/r03_gemm_bench2.log
FX_SPLIT_VARIANT=1 ROWS=8192 PREC=fp32s timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/r03_gemm_bench3.log 2>&1 || exit 6
echo "--- LDS-image split variant"; cat gpurun_out/r03_gemm_bench3.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -m gpu -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_split_test.log 2>&1
rc=$?; grep -E "PASS|FAIL|max \|err|^E " gpurun_out/r03_split_test.log | head -60; exit $rc
