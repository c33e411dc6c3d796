# A/B of the deferred MS-TCN weight-gradient schedule (knobs: FX_MSTCN_DEFER, FX_DEFER_SPLIT,
# FX_SIDE_PRIORITY), two alternating rounds on one box; prints ms/step per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 \
    > gpurun_out/ab_$name.json 2>/dev/null || return 1
  python -c "import json; d=json.load(open('gpurun_out/ab_$name.json')); print('$name', d['ms_per_step'], d['config']['tdu_segments'])"
}
for r in 1 2 3; do
  run off$r FX_MSTCN_DEFER=0 || exit 3
  run s8low_$r FX_DEFER_SPLIT=8 FX_SIDE_PRIORITY=low || exit 3
  run s8_$r FX_DEFER_SPLIT=8 || exit 3
  run s16low_$r FX_DEFER_SPLIT=16 FX_SIDE_PRIORITY=low || exit 3
done
