# Round 4: the fused layer kernel's backward launches alone vs with the side stream (FX_SIDE_STREAM=0 puts
# the deferred weight gradients on the caller's stream): per-kernel trace averages.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/frlbwd; rm -rf $O; mkdir -p $O
for x in FX_SIDE_STREAM=1 FX_SIDE_STREAM=0; do
  timeout -k 10 120 env $x rocprofv3 --kernel-trace --stats -d $O/p$x -o run --output-format csv -- python tools/frl_bwd_bench.py > $O/p$x.log 2>&1 || { tail -5 $O/p$x.log; exit 3; }
  grep "us/step" $O/p$x.log
  python - <<PY
import csv,glob
f=glob.glob('$O/p$x/**/run_kernel_stats.csv',recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r:-float(r['TotalDurationNs']))[:8]:
    print('$x', r['Calls'], round(float(r['AverageNs'])/1e3,1), r['Name'][:70])
PY
done
