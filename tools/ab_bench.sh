# A/B of an environment toggle on ONE box: alternate runs of bench.py (diagnostic)
# usage: AB="FACTMX_ROWSPLIT=0" bash tools/ab_bench.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2 3; do
  for side in A B; do
    if [ $side = A ]; then envs=""; else envs="$AB"; fi
    r=$(env $envs timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])") || exit 1
    echo "$side ($envs) $r ms/step"
  done
done
