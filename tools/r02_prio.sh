set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for pr in high normal low high normal; do
  FX_SIDE_PRIORITY=$pr timeout -k 10 200 python bench.py --steps 40 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/bench_pr$pr.json 2> gpurun_out/bench_pr$pr.err || exit 1
  echo "prio $pr: $(python -c "import json;d=json.loads(open('gpurun_out/bench_pr$pr.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
done
