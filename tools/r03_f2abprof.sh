set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in 1 0; do
  rm -rf gpurun_out/pc$v
  FX_X2Y_F2A_BWD=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pc$v -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/pc$v.log 2>&1 || exit 4
done
echo ok
