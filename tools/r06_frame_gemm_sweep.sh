# Round 6: tools/r06_frame_gemm_sweep.py under the planner's A/B knobs (one process each), twice.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  for e in "" "FX_GEMM_PERSIST=0" "FX_GEMM_GROUPM=0" "FX_GEMM_XCDPLANES=0" "FX_GEMM_WIDE=0" "FX_GEMM_W8=0" "FX_GEMM_PATH=tiled"; do
    env $e timeout -k 10 120 python tools/r06_frame_gemm_sweep.py 2>/dev/null >> gpurun_out/frame_gemm_sweep.txt || exit 1
  done
done
