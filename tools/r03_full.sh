# full GPU suite + smoke + phase timing of HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --maxfail 10 --timeout 300 --timeout-method thread > gpurun_out/r03_full_pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03_full_pytest.log | tail -15
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke2.log 2>&1 || exit 5
tail -1 gpurun_out/r03_smoke2.log
timeout -k 10 200 python tools/phase_times.py 2>&1 | grep -v amdgpu.ids | head -5
exit $rc
