# attention-over-T A/B (merge in launch vs separate, split sizes) + split-K reduce, then a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_attn_t.py tests/test_gpu_gemm.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ab.log; [ $rc -eq 0 ] || exit $rc
for mw in 256 512 1024; do
  for m in in launch; do
    echo "minwg=$mw merge=$m"
    FX_TATTN_MINWG=$mw FX_TATTN_MERGE=$m timeout -k 10 60 python tools/tattn_bench.py 4096 || exit 1
  done
done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --adam-steps 0 --no-cpu-baseline > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err
rc=$?; cut -c1-300 gpurun_out/bench_ab.json; exit $rc
