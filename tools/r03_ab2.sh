set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "FX_LAZY_READBACK=1 FX_X2Y_FUSED=1" "FX_LAZY_READBACK=0 FX_X2Y_FUSED=1" "FX_LAZY_READBACK=1 FX_X2Y_FUSED=0"; do
    env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-bf16 > gpurun_out/ab2.json 2>/dev/null || exit 4
    python -c "import json;d=json.loads(open('gpurun_out/ab2.json').read().splitlines()[-1]);print('$cfg', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], d['train_step_with_adam']['tdu_segments_after'])"
  done
done
