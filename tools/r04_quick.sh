# Round 4: model-level parity tests + two short bench runs (fixed-weight step and Adam leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/quick; rm -rf $O; mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_backward.py tests/test_gpu_parity.py tests/test_gpu_rccl.py} -x -q --timeout 250 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 2; }
tail -1 $O/t.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --no-dp-overhead --adam-steps 10 > $O/b$r.json 2>/dev/null || exit 5
  python -c "import json;d=json.loads(open('$O/b$r.json').read().splitlines()[-1]);print('run $r', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['tdu_segments'])"
done
