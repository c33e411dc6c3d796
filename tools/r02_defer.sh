# Deferred batched MS-TCN weight gradients: GPU parity (backward at the bench shape + GEMM/kernel suites),
# then an A/B of the bench step (FX_MSTCN_DEFER=0 = per-layer interleaved dW GEMMs) on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mstcn2.py tests/test_gpu_backward.py tests/test_gpu_parity.py tests/test_gpu_batch.py tests/test_gpu_gemm.py tests/test_gpu_kernels.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/defer_pytest.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/defer_pytest.log | tail -8; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  FX_MSTCN_DEFER=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/defer_off_$i.json 2>/dev/null || exit 3
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/defer_on_$i.json 2>/dev/null || exit 4
done
python - <<'PY'
import json
for t in ("off","on"):
    for i in (1,2):
        d=json.load(open(f"gpurun_out/defer_{t}_{i}.json")); print(t, i, d["ms_per_step"], d["value"], d["config"]["tdu_segments"])
PY
timeout -k 10 300 python bench.py --config breakfast --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/defer_bf.json 2>/dev/null && cut -c1-300 gpurun_out/defer_bf.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_defer -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_defer.log 2>&1
