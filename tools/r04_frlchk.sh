# Round 4: fused MS-TCN layer kernel check -- parity (pytest -k mstcn) and its trace-average duration in
# tools/frl_bench.py (forward layers) and in tools/frl_bench.py --bwd if present.  ENV passes knobs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/frlchk; rm -rf $O; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_backward.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 2; }
tail -1 $O/t.log
for x in ${VARIANTS:-0}; do
  rm -rf $O/p$x
  env $x timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p$x -o run --output-format csv -- python tools/frl_bench.py > $O/p.log 2>&1 || exit 3
  python - <<PY
import csv,glob
f=glob.glob('$O/p$x/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'frl_kernel' in r['Name']: print('$x', r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us', round(2*8192*256*1024/float(r['AverageNs'])/1e3,1), 'TF/s')
PY
done
