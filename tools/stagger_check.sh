set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
FX_GEMM_STAGGER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py -x -q -p no:cacheprovider > gpurun_out/st_t.log 2>&1; rc=$?; tail -2 gpurun_out/st_t.log; [ $rc -le 1 ] || exit $rc
for st in 0 1 0 1; do echo "== STAGGER=$st"; FX_GEMM_STAGGER=$st ROWS=8192 timeout -k 10 90 python tools/gemm_bench.py || exit 1; done
