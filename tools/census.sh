# GEMM shape census: FX_GEMM_LOG shape log + kernel trace of a 1-step bench (diagnostic; one stream, so
# the launch order of the log is the kernel order of the trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
rm -rf gpurun_out/census gpurun_out/gemm_log.txt
FX_SIDE_STREAM=0 FX_GEMM_LOG=gpurun_out/gemm_log.txt timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/census -o c \
  --output-format csv -- python bench.py --steps 1 --warmup 2 --no-cpu-baseline > gpurun_out/census.log 2>&1
