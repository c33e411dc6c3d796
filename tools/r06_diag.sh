# Round 6 GPU diagnostic of HEAD: targeted GPU tests, the default bench line, a kernel-trace profile of the
# bench (step map, idle gaps, top kernels, bench-vs-trace kernel times).  Every GPU step under its own time
# limit, chained; outputs under gpurun_out/r06diag.  TESTS=<pytest args> overrides the test selection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06diag; rm -rf $O; mkdir -p $O
T=${TESTS:-"tests/test_gpu_timeouts.py tests/test_gpu_x2y.py tests/test_gpu_decoder.py tests/test_gpu_attn_t.py"}
if [ "$T" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
  tail -3 $O/pytest.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
  tail -1 $O/bench.json | cut -c1-400
fi
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead ${BENCH_ARGS:-} > $O/prof.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 4; }
  # 3 warm-up + 1 calibration (event counts) + 10 timed steps = 14 steps in the profiled command
  python tools/kstats.py $(find $O/prof -name "*kernel_stats.csv") 14 40 > $O/kstats.txt
  python tools/step_map.py $(find $O/prof -name "*kernel_trace.csv") 10 > $O/step_map.txt
  python tools/gaps.py $(find $O/prof -name "*kernel_trace.csv") 3 terms_fwd_kernel > $O/gaps.txt
  python tools/r06_trace_groups.py $(find $O/prof -name "*kernel_trace.csv") $O/prof.json $O/trace_kernels.json > $O/trace_groups.txt
  head -3 $O/step_map.txt
fi
if [ "${STAMPS:-0}" = "1" ]; then
  timeout -k 10 300 python tools/r06_vloss_stamps.py > $O/vloss_stamps.txt 2>&1 || exit 5
  timeout -k 10 300 python tools/r06_host_ops.py > $O/host_ops.txt 2>&1 || exit 6
fi
echo done
