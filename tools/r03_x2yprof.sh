set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf gpurun_out/px0 gpurun_out/px1
FX_X2Y_FUSED=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/px0 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/px0.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/px1 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/px1.log 2>&1 || exit 5
echo ok
