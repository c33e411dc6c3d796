set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
ROWS=8192 PREC=${PRECS:-fp32,fp32s,bf16} timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/r03_gemm_bench2.log 2>&1 || { tail -20 gpurun_out/r03_gemm_bench2.log; exit 5; }
cat gpurun_out/r03_gemm_bench2.log
