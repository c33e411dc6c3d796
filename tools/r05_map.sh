# Round 5: kernel traces of the headline step at T=4096 and T=2048 (the fixed intercept per category),
# plus the shipped config's slow-GEMM census (FX_GEMM_LOG).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05map}; rm -rf $O; mkdir -p $O
for T in 4096 2048; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$T -o run --output-format csv -- python bench.py --T $T --steps 12 --warmup 4 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/p$T.log 2>&1 || exit 3
  echo "== T=$T"; python tools/step_map.py $(find $O/p$T -name "*kernel_trace.csv") 10
done
if [ "${CENSUS:-1}" = "1" ]; then
  FX_GEMM_LOG=$O/gemm_shipped.log timeout -k 10 200 python bench.py --config shipped --steps 4 --warmup 1 --adam-steps 0 --no-cpu-baseline --no-bf16 --no-dp-overhead > $O/shipped.json 2>&1 || exit 4
  echo "== shipped slow GEMMs"; python tools/gemm_slow.py $O/gemm_shipped.log 5
fi
