# Round 5 closing measurement of HEAD: the GPU test suite, the default bench line (with the CPU
# baseline), a kernel-trace profile and the step map of the headline config, and the PMC passes of the
# dominant kernel.  Every GPU step under its own time limit; outputs under gpurun_out/r05final.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r05final; rm -rf $O; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
  tail -3 $O/pytest_gpu.log
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
tail -1 $O/bench.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/prof.log 2>&1 || exit 4
python tools/kstats.py $(find $O/prof -name "*kernel_stats.csv") 13 30 > $O/kstats.txt
python tools/step_map.py $(find $O/prof -name "*kernel_trace.csv") 10 > $O/step_map.txt
head -3 $O/step_map.txt
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc_dominant.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 5; }
fi
echo done
