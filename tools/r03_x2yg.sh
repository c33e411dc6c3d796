set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_x2y.py tests/test_gpu_backward.py tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03_x2yg.log 2>&1 || { grep -E "^E |FAIL" gpurun_out/r03_x2yg.log | head; exit 2; }
tail -1 gpurun_out/r03_x2yg.log
CFGS="base" REPS="1 2 3" bash tools/r03_multi_ab.sh
