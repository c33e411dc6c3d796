set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for c in 0 128 64 160; do
  FX_SIDE_MAXWG=$c timeout -k 10 200 python bench.py --steps 20 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/bench_cap$c.json 2> gpurun_out/bench_cap$c.err || exit 1
  echo "cap $c: $(python -c "import json;d=json.loads(open('gpurun_out/bench_cap$c.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['value'])")"
done
