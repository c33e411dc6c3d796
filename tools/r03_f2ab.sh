set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_x2y.py tests/test_gpu_backward.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_f2ab.log 2>&1 || { grep -E "^E |FAIL" gpurun_out/r03_f2ab.log | head -20; exit 2; }
tail -1 gpurun_out/r03_f2ab.log
CFGS="base;FX_X2Y_F2A_BWD=0" REPS="1 2 3 4" bash tools/r03_multi_ab.sh
