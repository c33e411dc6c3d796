# GEMM kernels: correctness + A/B microbench + per-shape census of one bench step
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_gemm.py tests/test_gpu_kernels.py -q -p no:cacheprovider -x > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS:-libfactmx_prev.so libfactmx.so}" bash tools/ab_gemm.sh || exit $?
rm -f gpurun_out/gemm_log.txt
FX_GEMM_LOG=$PWD/gpurun_out/gemm_log.txt timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/census -o c --output-format csv -- python bench.py --steps 1 --warmup 2 --no-cpu-baseline > gpurun_out/census.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline
