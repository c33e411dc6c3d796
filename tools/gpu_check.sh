# Full GPU pass: parity tests, smoke, bench (HAViD + Breakfast lines), kernel-trace profile.
# Stops at the first crash/timeout (pytest exit 1 = ordinary test failures, still safe to continue).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG="${TAG:-run}"
TESTS="${TESTS:-tests}"
timeout -k 10 1000 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu_$TAG.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke exit $rc"; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cat gpurun_out/bench_$TAG.json; tail -3 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --config breakfast --steps 10 --warmup 3 > gpurun_out/bench_bf_$TAG.json 2> gpurun_out/bench_bf_$TAG.err
rc=$?; echo "bench breakfast exit $rc"; cat gpurun_out/bench_bf_$TAG.json; tail -3 gpurun_out/bench_bf_$TAG.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof exit $rc"; tail -1 gpurun_out/prof_$TAG.log
exit $rc
