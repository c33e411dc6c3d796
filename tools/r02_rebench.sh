set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-bf16 > gpurun_out/rb.json 2>/dev/null || exit 4
python -c "import json; d=json.load(open('gpurun_out/rb.json')); print('havid', d['ms_per_step'], d['value'], d['train_step_with_adam']['ms_per_step'])"
done
nproc; cat /proc/loadavg
