# Round 6 closing measurement of HEAD: the GPU test suite, the default bench line (with the CPU baseline), the
# T=2048, shipped-yaml and Breakfast lines, a kernel-trace profile of the headline config (step map, idle
# gaps, top kernels, per-kernel trace averages for bench.py's trace-basis rooflines) and the PMC passes of the
# dominant kernel.  Every GPU step under its own time limit; outputs under gpurun_out/r06final.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06final; rm -rf $O; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
  tail -1 $O/pytest_gpu.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/prof.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 4; }
# 3 warm-up + 1 calibration (event counts) + 10 timed steps = 14 steps in the profiled command
python tools/kstats.py $(find $O/prof -name "*kernel_stats.csv") 14 40 > $O/kstats.txt
# the step map over the last 8 step periods: the first timed step carries bench.py's sampled kernel-event pairs
# (hipExtLaunchKernel under the tracer: ~45 ms of host time in that one step), which is not the step's idle
python tools/step_map.py $(find $O/prof -name "*kernel_trace.csv") 8 > $O/step_map.txt
python tools/gaps.py $(find $O/prof -name "*kernel_trace.csv") 3 terms_fwd_kernel > $O/gaps.txt
python tools/r06_trace_groups.py $(find $O/prof -name "*kernel_trace.csv") $O/prof.json $O/trace_kernels.json > $O/trace_groups.txt
cp $O/trace_kernels.json profiles/r06_trace_kernels.json
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
tail -1 $O/bench.json | cut -c1-300
if [ "${LINES:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --T 2048 --no-dp-overhead > $O/bench_T2048.json 2> $O/bench_T2048.err || exit 5
  timeout -k 10 600 python bench.py --config shipped --no-bf16 --no-dp-overhead > $O/bench_shipped.json 2> $O/bench_shipped.err || exit 6
  timeout -k 10 600 python bench.py --config breakfast --no-bf16 --no-dp-overhead > $O/bench_breakfast.json 2> $O/bench_breakfast.err || exit 7
fi
if [ "${PMC:-1}" = "1" ]; then
  bash tools/pmc_dominant.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 8; }
fi
echo done
