# SQ counters for one GEMM shape of tools/gemm_bench.py (diagnostic; counters in their own passes)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/pmc_gemm
mkdir -p $OUT
export CASE="${CASE:-conv fwd}"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/p1 -o p1 --output-format csv -- python tools/gemm_bench.py > $OUT/p1.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o p2 --output-format csv -- python tools/gemm_bench.py > $OUT/p2.log 2>&1
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/p3 -o p3 --output-format csv -- python tools/gemm_bench.py > $OUT/p3.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/t -o t --output-format csv -- python tools/gemm_bench.py > $OUT/t.log 2>&1
echo done
