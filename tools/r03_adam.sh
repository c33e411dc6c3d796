set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for a in "" "--no-bf16"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline $a > gpurun_out/adam.json 2>/dev/null || exit 4
    python -c "import json;d=json.loads(open('gpurun_out/adam.json').read().splitlines()[-1]);print('args[$a]', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], d['train_step_with_adam']['tdu_segments_after'])"
  done
done
