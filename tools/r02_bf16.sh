set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_gemm.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pytest_bf16.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/pytest_bf16.log | tail -25; [ $rc -eq 0 ] || exit $rc
LD_LIBRARY_PATH=fact-clip_amd/factmx/_lib timeout -k 10 120 tools/gemm_sweep
