# Round 4: same-box A/B of environment knobs on the bench step: VARIANTS="A=1 B=2 ..." (each a space-free
# env assignment, "none" for the default), 3 rounds alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/envab; rm -rf $O; mkdir -p $O
for r in $(seq ${ROUNDS:-3}); do for x in $VARIANTS; do
  e=$x; [ "$x" = none ] && e=FX_NOOP=1
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --no-dp-overhead --adam-steps 10 ${BENCH_ARGS:-} > $O/b.json 2>/dev/null || exit 5
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print('$x', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], d['roofline']['avg_launch_ms'])"
done; done
