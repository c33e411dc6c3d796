"""Diagnostic: the fused MS-TCN layer kernel (frl_kernel) alone: a 10-layer F=256 MS-TCN forward
(in_map off) on 2 x 4096 rows, timed with HIP events (python tools/frl_bench.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402
from factmx.models.basic import MSTCN  # noqa: E402


def main():
    torch.manual_seed(0)
    mod = MSTCN(256, 256, 256, 10, dropout=0.0, ln=False, in_map=False).cuda().eval()
    x = torch.randn(8192, 256, device="cuda")
    with torch.no_grad():
        for _ in range(3):
            fxf.mstcn(mod, x, T=4096, nvid=2)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        n = 20
        for _ in range(n):
            fxf.mstcn(mod, x, T=4096, nvid=2)
        b.record()
        torch.cuda.synchronize()
    us = a.elapsed_time(b) / n * 1e3
    fl = 2.0 * 8192 * 256 * 1024 * 10
    print(f"MS-TCN fwd 10 layers: {us:.1f} us/stack, {fl / us / 1e6:.1f} TF/s incl. in/out maps")


if __name__ == "__main__":
    main()
