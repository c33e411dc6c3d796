# Round-3 first GPU check: full GPU suite (no -x: see every failure), smoke, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --maxfail 15 --timeout 300 --timeout-method thread > gpurun_out/r03_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_pytest.log | tail -25
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit 5
tail -1 gpurun_out/r03_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || exit 3
cut -c1-600 gpurun_out/r03_bench.json
exit $rc
