# Round-6 diagnostic: the GEMM census of a bench run (census build of the library, built in-tree with
#   make -C fact-clip_amd/csrc OBJDIR=build_diag OUT=../factmx/_lib/diag/libfactmx.so CXXFLAGS="... -DFX_GEMM_CENSUS")
# joined with the kernel trace of the same run.  Outputs under gpurun_out/r06census.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06census; rm -rf $O; mkdir -p $O
export FACTMX_LIB=$GRAFT_REPO_ROOT/fact-clip_amd/factmx/_lib/diag/libfactmx.so
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/bench.json 2> $O/census.txt || { tail -5 $O/census.txt; exit 3; }
python tools/r06_gemm_census.py $O/census.txt $(find $O/prof -name "*kernel_trace.csv") > $O/gemm_census.txt
head -50 $O/gemm_census.txt
