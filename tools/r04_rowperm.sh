# Round 4: A/B of the dilation-aware row-tile -> XCD mapping of the conv GEMMs (FX_GEMM_ROWPERM):
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) and kernel-trace durations of the dominant kernel,
# then a short bench line (roofline + roofline_attention incl. the X2Y cores).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/rowperm
rm -rf $OUT; mkdir -p $OUT
for rp in 1 0; do
  for set in FETCH_SIZE WRITE_SIZE; do
    FX_GEMM_ROWPERM=$rp timeout -s KILL 240 rocprofv3 --pmc $set -d $OUT/rp${rp}_$set -o p --output-format csv -- \
      python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-bf16 --adam-steps 0 --no-dp-overhead > $OUT/rp${rp}_$set.log 2>&1 || { echo "pmc $rp $set failed"; tail -5 $OUT/rp${rp}_$set.log; exit 1; }
  done
  mkdir -p $OUT/pm$rp; cp -r $OUT/rp${rp}_FETCH_SIZE $OUT/pm$rp/p1; cp -r $OUT/rp${rp}_WRITE_SIZE $OUT/pm$rp/p2
  python tools/pmc_dominant.py $OUT/pm$rp "gemm_f32_wide8_kernel<1, 0, 0>" > $OUT/pmc_rp$rp.json
  FX_GEMM_ROWPERM=$rp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt$rp -o run --output-format csv -- \
    python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-bf16 --adam-steps 0 --no-dp-overhead > $OUT/kt$rp.log 2>&1 || { echo "trace $rp failed"; exit 1; }
done
for rp in 1 0; do
  python -c "import json;d=json.load(open('$OUT/pmc_rp$rp.json'));print('rowperm $rp hbm MB/launch', round(d['hbm_bytes_per_launch']/1e6,2), 'fetch', round(d['fetch_bytes_per_launch']/1e6,2))"
  grep "gemm_f32_wide8_kernel<1, 0, 0>" $OUT/kt$rp/run_kernel_stats.csv | cut -d, -f1-4
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bf16 > $OUT/bench.json 2> $OUT/bench.err || exit 5
python -c "import json;d=json.loads(open('$OUT/bench.json').read().splitlines()[-1]);print(d['ms_per_step'], d['roofline']['frac']);[print(k, v and (v['frac'], v['avg_launch_ms'], v['launches'])) for k,v in d['roofline_attention'].items()]; print(d['dp_schedule'])"
