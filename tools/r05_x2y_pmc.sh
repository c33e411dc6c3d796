# Round 5: FETCH_SIZE / WRITE_SIZE passes (separate runs) over the X2Y bench (tools/r05_x2y_bench.py, the
# headline shapes), per direction; per-launch HBM bytes of the X2Y core kernels summed per bracket ->
# gpurun_out/r05_pmc_x2y.json (bench.py fills roofline_attention.x2y_*.traffic from profiles/ copy)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for d in a2f f2a; do
  OUT=gpurun_out/pmc_x2y_$d; rm -rf $OUT; mkdir -p $OUT
  i=0
  for set in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p$i -o p$i --output-format csv -- \
      python tools/r05_x2y_bench.py $d 8 > $OUT/p$i.log 2>&1 || { echo "pass $d $set failed"; tail -5 $OUT/p$i.log; exit 1; }
  done
done
python tools/r05_x2y_pmc.py > gpurun_out/r05_pmc_x2y.json && cat gpurun_out/r05_pmc_x2y.json
