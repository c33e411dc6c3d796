# MS-TCN dZ GEMM on the forward-packed transposed 1x1 weight: parity subset + bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_backward.py tests/test_gpu_decoder.py tests/test_gpu_parity.py tests/test_gpu_batch.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/wpt_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/wpt_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-bf16 > gpurun_out/wpt.json 2>/dev/null || exit 4
python -c "import json; d=json.load(open('gpurun_out/wpt.json')); print('havid', d['ms_per_step'], d['value'], d['train_step_with_adam']['ms_per_step'])"
done
cat /proc/loadavg
