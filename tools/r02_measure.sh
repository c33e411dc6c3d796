set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err && cut -c1-3000 gpurun_out/r02_bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r02 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline > gpurun_out/prof_r02.log 2>&1 &&
bash tools/pmc_dominant.sh > gpurun_out/pmc.log 2>&1
echo "exit $?"
