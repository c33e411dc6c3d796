# Round 4: XCD-aware row-tile order of the fused MS-TCN layer kernel (FX_FRL_XCD 0 round robin /
# 1 contiguous runs / 2 runs following the conv taps): parity, the stack alone, PMC fetch, whole step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/frlx; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "mstcn" -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 2; }
tail -1 $O/t.log
for x in 0 1 2 0 1 2; do FX_FRL_XCD=$x timeout -k 10 120 python -u tools/frl_bench.py 2>&1 | grep -v amdgpu | sed "s/^/xcd=$x /" || exit 3; done
for x in 0 2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    FX_FRL_XCD=$x timeout -s KILL 90 rocprofv3 --pmc $c -d $O/pm$x$c -o p --output-format csv -- python tools/frl_bench.py > $O/pm$x$c.log 2>&1 || { echo "pmc $x $c failed"; exit 4; }
  done
done
for r in 1 2; do for x in 0 2; do
  FX_FRL_XCD=$x timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --no-dp-overhead --adam-steps 10 > $O/b$x$r.json 2>/dev/null || exit 5
  python -c "import json;d=json.loads(open('$O/b$x$r.json').read().splitlines()[-1]);f=d['roofline_fused_layer'];print('xcd=$x', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], f['avg_launch_ms'], f['frac'])"
done; done
