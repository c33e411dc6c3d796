# Round 5: GEMM census of the headline step (FX_GEMM_LOG joined with a kernel trace): time per GEMM shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05cen}; rm -rf $O; mkdir -p $O
FX_GEMM_LOG=$O/gemm.log timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p -o run --output-format csv -- python bench.py --config ${CFG:-havid} --steps 4 --warmup 1 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/p.log 2>&1 || exit 3
python tools/gemm_census.py $O/gemm.log $(find $O/p -name "*kernel_trace.csv")
