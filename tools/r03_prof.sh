# Round-3 profile of HEAD: parity test fix, kernel-trace stats of the bench line, op-group timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03_parity.log 2>&1 || { tail -30 gpurun_out/r03_parity.log; exit 1; }
tail -1 gpurun_out/r03_parity.log
rm -rf gpurun_out/prof_r03
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_r03.log 2>&1 || exit 4
timeout -k 10 300 python tools/op_bench.py > gpurun_out/op_bench_r03.log 2>&1 || exit 5
tail -40 gpurun_out/op_bench_r03.log
