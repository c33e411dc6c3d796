set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for r in 1 2; do
for cfg in "10 3" "10 6" "20 5" "30 3"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/wu.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/wu.json')); print('steps $1 warmup $2', d['ms_per_step'])"
done
done
