# Round-3: ntoken-75 model test, the shipped-yaml bench line, the T=2048 (configs[1]) line with its bf16 mode
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py -m gpu -x -v -p no:cacheprovider -k ntoken75 --timeout 300 --timeout-method thread > gpurun_out/r03_nt75.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|^E " gpurun_out/r03_nt75.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config shipped > gpurun_out/r03_bench_shipped.json 2> gpurun_out/r03_bench_shipped.err || { tail -20 gpurun_out/r03_bench_shipped.err; exit 3; }
cut -c1-400 gpurun_out/r03_bench_shipped.json
timeout -k 10 400 python bench.py --T 2048 > gpurun_out/r03_bench_T2048.json 2> gpurun_out/r03_bench_T2048.err || { tail -20 gpurun_out/r03_bench_T2048.err; exit 4; }
cut -c1-300 gpurun_out/r03_bench_T2048.json
ROWS=8192 PREC=fp32,bf16 timeout -k 10 120 python tools/gemm_bench.py > gpurun_out/r03_gemm_bench.log 2>&1 || exit 5
cat gpurun_out/r03_gemm_bench.log
