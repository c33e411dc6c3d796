# A/B of an env knob on the default bench line: alternating runs (KNOB=name, A=value, B=value)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for r in ${REPS:-1 2 3}; do
  for val in $A $B; do
    env $KNOB=$val timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --adam-steps 0 > gpurun_out/ab_${val}_$r.json 2>/dev/null || exit 4
    python -c "import json;d=json.loads(open('gpurun_out/ab_${val}_$r.json').read().splitlines()[-1]);print('$KNOB=$val', d['ms_per_step'])"
  done
done
