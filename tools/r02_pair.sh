# MS-TCN++ conv pair as one batch-2 launch: parity subset, Breakfast bench, default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mstcn2.py tests/test_gpu_backward.py tests/test_gpu_gemm.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_kernels.py tests/test_gpu_long.py tests/test_gpu_vloss.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pair_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/pair_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config breakfast --no-cpu-baseline > gpurun_out/pair_bf.json 2>/dev/null || exit 3
python -c "import json; d=json.load(open('gpurun_out/pair_bf.json')); print('breakfast', d['ms_per_step'], d['value'], d['roofline']['frac'], d['bf16_mode']['ms_per_step'])"
timeout -k 10 400 python bench.py > gpurun_out/bench_sampled.json 2> gpurun_out/bench_sampled.err || exit 4
python -c "import json; d=json.load(open('gpurun_out/bench_sampled.json')); print('havid', d['ms_per_step'], d['value'], d['roofline']['frac'], d['train_step_with_adam']['ms_per_step'], d['bf16_mode']['ms_per_step'], d['cpu_baseline']['value'], d['step_mfma_frac'])"
