set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x2y.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03_x2y_test.log 2>&1 || { grep -E "^E |FAIL" gpurun_out/r03_x2y_test.log | head -20; exit 2; }
tail -1 gpurun_out/r03_x2y_test.log
timeout -k 10 200 python tools/host_ops.py > gpurun_out/r03_host_ops.log 2>&1 || { tail -20 gpurun_out/r03_host_ops.log; exit 3; }
head -3 gpurun_out/r03_host_ops.log
FX_X2Y_FUSED=0 timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-bf16 --adam-steps 0 > gpurun_out/r03_b_x2y0.json 2>/dev/null || exit 4
timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-bf16 --adam-steps 0 > gpurun_out/r03_b_x2y1.json 2>/dev/null || exit 5
FX_X2Y_FUSED=0 timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-bf16 --adam-steps 0 > gpurun_out/r03_b_x2y0b.json 2>/dev/null || exit 6
timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline --no-bf16 --adam-steps 0 > gpurun_out/r03_b_x2y1b.json 2>/dev/null || exit 7
for f in x2y0 x2y1 x2y0b x2y1b; do python -c "import json;d=json.loads(open('gpurun_out/r03_b_$f.json').read().splitlines()[-1]);print('$f',d['ms_per_step'])"; done
