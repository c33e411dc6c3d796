# Run-to-run spread of the default bench line on one box (5 runs), host load at the end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-bf16 > gpurun_out/spread_$i.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/spread_$i.json')); print('run $i', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
cat /proc/loadavg
