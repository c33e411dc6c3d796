"""Round 5: the frame-level linear shapes of the step alone (y = x W^T + b through factmx.functional.linear,
the wide GEMM kernels), HIP-event timed: avg us, TF/s, fraction of the f32 MFMA peak.

python tools/r05_linear_sweep.py [rows]"""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "fact-clip_amd")]
from factmx import functional as fxf  # noqa: E402

PEAK = 157.3
M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
for K, N in [(256, 256), (256, 512), (512, 256), (512, 512), (512, 1024), (1024, 512), (512, 3072), (3072, 512),
             (2048, 256), (768, 256)]:
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") * K ** -0.5
    b = torch.zeros(N, device="cuda")
    with torch.no_grad():
        for _ in range(5):
            fxf.linear(x, w, b)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(30):
            fxf.linear(x, w, b)
        e.record()
        torch.cuda.synchronize()
    us = s.elapsed_time(e) * 1e3 / 30
    tf = 2.0 * M * N * K / us / 1e6
    print(f"M {M} K {K:5d} N {N:5d}: {us:7.1f} us  {tf:6.1f} TF/s  {tf / PEAK:.3f}", flush=True)
