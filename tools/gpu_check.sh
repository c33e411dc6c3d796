set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 500 > gpurun_out/pytest_gpu3.log 2>&1; echo "pytest exit $?"
tail -4 gpurun_out/pytest_gpu3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo smoke ok || echo smoke FAIL
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err && echo bench ok || echo bench FAIL
cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof1.log 2>&1 && echo prof ok || echo prof FAIL
