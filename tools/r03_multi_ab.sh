# interleaved A/B over several env settings (CFGS: ';'-separated, each a space-separated env list or "base")
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
IFS=';' read -ra C <<< "$CFGS"
for r in ${REPS:-1 2 3}; do
  for cfg in "${C[@]}"; do
    e=$cfg; [ "$cfg" = "base" ] && e=""
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --adam-steps 0 > gpurun_out/mab.json 2>/dev/null || exit 4
    python -c "import json;d=json.loads(open('gpurun_out/mab.json').read().splitlines()[-1]);print('$cfg', d['ms_per_step'])"
  done
done
