# PMC passes over a short bench run, one counter group per rocprofv3 pass (never combined with
# trace domains): HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes) and SQ issue/stall
# counters, averaged per launch of the dominant kernel -> gpurun_out/pmc_dominant.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_dom
rm -rf $OUT; mkdir -p $OUT
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $set -d $OUT/p$i -o p$i --output-format csv -- \
    python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-bf16 > $OUT/p$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_dominant.py $OUT "${KERNEL:-frl_kernel}" > gpurun_out/pmc_dominant.json
# the dilated-conv GEMM (the dominant kernel before the fused layer became the default)
python tools/pmc_dominant.py $OUT "gemm_f32_wide8_kernel<1, 0, 0>" > gpurun_out/pmc_conv_gemm.json
cat gpurun_out/pmc_dominant.json
# the same FETCH/WRITE passes, averaged over the attention-over-T kernels
# (head dim 32: the register-resident kernels, round 5)
python tools/pmc_dominant.py $OUT "tattn_fwd32_kernel" > gpurun_out/r05_pmc_tattn_fwd.json
python tools/pmc_dominant.py $OUT "tattn_bwd32_kernel" > gpurun_out/r05_pmc_tattn_bwd.json
