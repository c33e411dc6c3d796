# Plane-per-XCD tile mapping (FX_GEMM_XCDPLANES): parity subset, dW micro-benchmark and bench A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
[ "${SKIP_TESTS:-0}" = "1" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_gemm.py tests/test_gpu_mstcn2.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/xcd_pytest.log 2>&1
rc=$?; [ "${SKIP_TESTS:-0}" = "1" ] || { tail -2 gpurun_out/xcd_pytest.log; [ $rc -eq 0 ] || exit $rc; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "planes off:"; FX_GEMM_XCDPLANES=0 timeout -k 10 120 python tools/cols_bench.py || exit 3
  echo "planes on:"; timeout -k 10 120 python tools/cols_bench.py || exit 3
fi
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 30 --warmup 3 --adam-steps 0 --no-cpu-baseline --no-bf16 \
    > gpurun_out/xab_$name.json 2>/dev/null || return 1
  python -c "import json; d=json.load(open('gpurun_out/xab_$name.json')); print('$name', d['ms_per_step'])"
}
for r in 1 2 3 4; do
  run on$r || exit 4
  run off$r FX_GEMM_XCDPLANES=0 || exit 4
done
