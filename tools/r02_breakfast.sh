set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_bk.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_bk.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config breakfast --steps 10 --warmup 3 --no-cpu-baseline --adam-steps 0 > gpurun_out/bench_bk.json 2> gpurun_out/bench_bk.err
rc=$?; cut -c1-250 gpurun_out/bench_bk.json; tail -2 gpurun_out/bench_bk.err; exit $rc
