# Round-2 closing measurement: full GPU suite, smoke, the default bench line (CPU baseline + bf16
# mode), its kernel-trace stats, the PMC passes of the dominant kernel / attention, the Breakfast line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final_pytest.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/final_pytest.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit 5
tail -1 gpurun_out/final_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 3
cut -c1-300 gpurun_out/final_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_final.log 2>&1 || exit 4
bash tools/pmc_dominant.sh > gpurun_out/pmc_final.log 2>&1 || exit 6
timeout -k 10 400 python bench.py --config breakfast > gpurun_out/final_bench_bf.json 2> gpurun_out/final_bench_bf.err || exit 7
cut -c1-300 gpurun_out/final_bench_bf.json
