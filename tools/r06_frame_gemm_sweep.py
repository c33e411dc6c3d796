"""Diagnostic: the frame-level linear GEMMs of the headline step alone (fxf.linear forward, HIP events), one
line per shape: the SCA K/V projection of every decoder layer (8192 x 3072 x 512), the X2Y input projections
(8192 x 512 x 512) and the MS-TCN 1x1 maps (8192 x 256 x 256).  Run under different FX_GEMM_* knobs (one
process each: the knobs are read once) to compare the planner's tile / order choices per shape.
    python tools/r06_frame_gemm_sweep.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402

PEAK = 157.3


def timeit(fn, iters=40):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    torch.manual_seed(0)
    out = []
    for M, N, K in ((8192, 3072, 512), (8192, 512, 512), (8192, 256, 256), (8192, 512, 256), (8192, 256, 512)):
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda") * K ** -0.5
        b = torch.randn(N, device="cuda")
        with torch.no_grad():
            us = timeit(lambda: fxf.linear(x, w, b))
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        out.append(f"{M}x{N}x{K} {us:7.1f} us {tf:6.1f} TF/s {tf / PEAK:.3f}")
    tag = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("FX_GEMM")) or "default"
    print(f"[{tag}] " + " | ".join(out), flush=True)


if __name__ == "__main__":
    main()
