"""Diagnostic: a 10-layer F=256 MS-TCN forward + backward (fused layer kernel in both directions) on
2 x 4096 rows, timed with HIP events; run under rocprofv3 --kernel-trace --stats for per-kernel
durations (python tools/frl_bwd_bench.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402
from factmx.dp import FlatGradReducer  # noqa: E402
from factmx.models.basic import MSTCN  # noqa: E402


def main():
    torch.manual_seed(0)
    mod = MSTCN(256, 256, 256, 10, dropout=0.0, ln=False, in_map=True).cuda().train()
    FlatGradReducer(mod.parameters())     # uniformly strided gradients: the deferred batched dW path
    x = torch.randn(8192, 256, device="cuda", requires_grad=True)
    g = torch.randn(8192, 256, device="cuda")

    def step():
        y = fxf.mstcn(mod, x, T=4096, nvid=2)
        y.backward(g)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    n = 20
    for _ in range(n):
        step()
    b.record()
    torch.cuda.synchronize()
    print(f"MS-TCN fwd+bwd 10 layers: {a.elapsed_time(b) / n * 1e3:.1f} us/step")


if __name__ == "__main__":
    main()
