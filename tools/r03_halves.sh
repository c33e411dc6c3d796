set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_mstcn2.py tests/test_gpu_kernels.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_halves_test.log 2>&1 || { grep -E "^E |FAIL" gpurun_out/r03_halves_test.log | head -20; exit 2; }
tail -1 gpurun_out/r03_halves_test.log
KNOB=FX_MSTCN_DW_HALVES A=0 B=1 REPS="1 2 3 4" bash tools/r03_ab.sh
