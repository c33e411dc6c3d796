# Quick GPU check: the given tests (TESTS), a bench line and a kernel-trace profile (TAG names outputs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG="${TAG:-chk}"
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_backward.py} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; grep -E "FAILED|passed|failed|Error" gpurun_out/pytest_$TAG.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/bench_$TAG.json 2>/dev/null || exit 3
cut -c1-260 gpurun_out/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 > gpurun_out/prof_$TAG.log 2>&1
