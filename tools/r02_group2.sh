set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_decoder.py tests/test_gpu_kernels.py tests/test_gpu_batch.py tests/test_gpu_backward.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_grp.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_grp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline > gpurun_out/bench_grp.json 2> gpurun_out/bench_grp.err
rc=$?; cut -c1-200 gpurun_out/bench_grp.json; [ $rc -eq 0 ] || exit $rc
bash tools/census.sh
