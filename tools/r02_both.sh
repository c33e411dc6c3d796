# Parity subset (TESTS) + both bench lines (HAViD default shape, Breakfast), 2 runs each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/both_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/both_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --config breakfast --steps 20 --no-cpu-baseline --no-bf16 > gpurun_out/both_bf.json 2>/dev/null || exit 3
  python -c "import json; d=json.load(open('gpurun_out/both_bf.json')); print('breakfast', d['ms_per_step'], d['value'])"
  timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-bf16 > gpurun_out/both_hv.json 2>/dev/null || exit 4
  python -c "import json; d=json.load(open('gpurun_out/both_hv.json')); print('havid', d['ms_per_step'], d['value'])"
done
cat /proc/loadavg
