# Round 4: stage-pair synchronisation of the fused MS-TCN layer kernel (FX_FRL_PAIR 0/1): parity, the
# stack alone, the whole step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/frlp; rm -rf $O; mkdir -p $O
for x in 1 0; do
  FX_FRL_PAIR=$x timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "mstcn" -x -q --timeout 200 --timeout-method thread > $O/t$x.log 2>&1 || { tail -20 $O/t$x.log; exit 2; }
  tail -1 $O/t$x.log
done
for x in 0 1 0 1; do FX_FRL_PAIR=$x timeout -k 10 120 python -u tools/frl_bench.py 2>&1 | grep -v amdgpu | sed "s/^/pair=$x /" || exit 3; done
for r in 1 2; do for x in 0 1; do
  FX_FRL_PAIR=$x timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 --no-dp-overhead --adam-steps 10 > $O/b$x$r.json 2>/dev/null || exit 5
  python -c "import json;d=json.loads(open('$O/b$x$r.json').read().splitlines()[-1]);f=d['roofline_fused_layer'];print('pair=$x', d['ms_per_step'], d['train_step_with_adam']['ms_per_step'], f['avg_launch_ms'], f['frac'])"
done; done
