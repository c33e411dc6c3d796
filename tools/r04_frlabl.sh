# Round 4 diagnostic: timing ablations of the fused MS-TCN layer kernel (FX_FRL_ABLATE bits, WRONG
# results -- timing only): which operand stream or synchronisation holds it below the MFMA rate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/frlabl; rm -rf $O; mkdir -p $O
for x in 0 1 2 4 8 15 0; do
  rm -rf $O/p$x
  FX_FRL_ABLATE=$x timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p$x -o run --output-format csv -- python tools/frl_bench.py > $O/p$x.log 2>&1 || exit 3
  python - <<PY
import csv,glob
f=glob.glob('$O/p$x/**/run_kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'frl_kernel' in r['Name']: print('ablate=$x', r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us', round(2*8192*256*1024/float(r['AverageNs'])/1e3,1), 'TF/s')
PY
done
