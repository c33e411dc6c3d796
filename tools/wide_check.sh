# Forced-wide-tile GEMM correctness + A/B microbench of 64x64 vs 128x64 tiles (diagnostic)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
FX_GEMM_WIDE=1 FX_GEMM_W8=${W8:-1} timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py \
  tests/test_gpu_decoder.py -x -q -p no:cacheprovider --timeout 100 --timeout-method thread > gpurun_out/wide_t.log 2>&1
rc=$?; tail -5 gpurun_out/wide_t.log; [ $rc -le 1 ] || exit $rc
for w in "0 1" "1 0" "1 1"; do
  set -- $w
  echo "== WIDE=$1 W8=$2"
  FX_GEMM_WIDE=$1 FX_GEMM_W8=$2 ROWS=8192 timeout -k 10 90 python tools/gemm_bench.py || exit $?
done > gpurun_out/wide_b.log 2>&1
rc=$?; cat gpurun_out/wide_b.log; exit $rc
