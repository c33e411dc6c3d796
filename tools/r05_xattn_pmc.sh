# Round 5: FETCH_SIZE and WRITE_SIZE (separate passes) of the cross-attention projection GEMMs alone,
# averaged per dispatch of the GEMM kernel -> gpurun_out/r05_pmc_{kvproj,x2yproj}.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for which in kv x2y; do
  OUT=gpurun_out/pmc_$which; rm -rf $OUT; mkdir -p $OUT
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o p$i --output-format csv -- \
      python tools/r05_xattn_pmc.py $which > $OUT/p$i.log 2>&1 || { echo "pass $which $set failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
  name=$([ $which = kv ] && echo kvproj || echo x2yproj)
  python tools/pmc_dominant.py $OUT gemm_f32_wide > gpurun_out/r05_pmc_$name.json
  cat gpurun_out/r05_pmc_$name.json
done
