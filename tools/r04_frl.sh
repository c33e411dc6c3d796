# Round 4: the fused MS-TCN layer kernel with fragment-packed weights: correctness (fused and unfused
# paths vs fp64), the stack alone (tools/frl_bench.py), and the full step A/B (FX_MSTCN_FUSED_LAYERS).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/frl
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_decoder.py tests/test_gpu_decoder_ext.py tests/test_gpu_backward.py -x -q --timeout 250 --timeout-method thread > gpurun_out/frl/t.log 2>&1; rc=$?
tail -3 gpurun_out/frl/t.log; [ $rc -eq 0 ] || exit 3
for f in 0 1; do FX_MSTCN_FUSED_LAYERS=$f timeout -k 10 120 python -u tools/frl_bench.py 2>&1 | grep -v amdgpu | sed "s/^/fused=$f /" || exit 4; done
for r in 1 2; do for f in 0 1; do
  FX_MSTCN_FUSED_LAYERS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --no-dp-overhead --adam-steps 10 > gpurun_out/frl/b$f$r.json 2>/dev/null || exit 5
  python -c "import json;d=json.loads(open('gpurun_out/frl/b$f$r.json').read().splitlines()[-1]);print('fused=$f', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['config']['tdu_segments'])"
done; done
