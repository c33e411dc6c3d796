# Quick GPU pass: the given tests (TESTS), then a short bench (+ optional kernel-trace profile when PROF=1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG="${TAG:-q}"
TESTS="${TESTS:-tests}"
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "FAILED|passed|failed|error" gpurun_out/pytest_$TAG.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench exit $rc"; cut -c1-400 gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "prof exit $rc"
fi
exit $rc
