# GEMM shape census of HEAD (single stream so log order == kernel order) + summary
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/census.sh || exit 1
python tools/gemm_census.py gpurun_out/gemm_log.txt gpurun_out/census/c_kernel_trace.csv > gpurun_out/census_r03.txt 2>&1 || exit 2
head -45 gpurun_out/census_r03.txt
