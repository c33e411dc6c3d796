# Cost of the live HIP-event timing inside the timed region: every timed step vs only the first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 \
    > gpurun_out/pab_$name.json 2>/dev/null || return 1
  python -c "import json; d=json.load(open('gpurun_out/pab_$name.json')); print('$name', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches'])"
}
for r in 1 2 3; do
  run all$r || exit 4
  run one$r FX_BENCH_PROF_STEPS=1 || exit 4
  run none$r FX_BENCH_PROF_STEPS=0 || exit 4
done
