# Segment-level GEMM shapes on the tiled vs direct kernel (tools/r06_seg_gemm.py, SWEEP=1: the crossover) and,
# with IID=1, the iid stress bench line.  Outputs under gpurun_out/r06iid.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06iid; mkdir -p $O
for p in ${PATHS:-planner tiled direct}; do
  if [ $p = planner ]; then timeout -k 10 180 python tools/r06_seg_gemm.py > $O/seg${SWEEP}_$p.txt 2>&1 || exit 3
  else FX_GEMM_PATH=$p timeout -k 10 180 python tools/r06_seg_gemm.py > $O/seg${SWEEP}_$p.txt 2>&1 || exit 3; fi
done
cat $O/seg${SWEEP}_*.txt | grep -v amdgpu.ids
if [ "${IID:-0}" = "1" ]; then
  timeout -k 10 900 python bench.py --data iid --steps 3 --warmup 1 --adam-steps 0 --no-bf16 --no-dp-overhead > $O/bench_iid.json 2> $O/bench_iid.err || { tail -20 $O/bench_iid.err; exit 4; }
  tail -1 $O/bench_iid.json | cut -c1-400
fi
