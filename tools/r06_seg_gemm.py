"""Segment-level GEMM shapes (TDU blocks: S ~ 50-130 segments per video, 2 videos) on the tiled 64x64 kernel
vs the direct kernel (diagnostic).  Run once per path:

FX_GEMM_PATH=tiled  python tools/r06_seg_gemm.py
FX_GEMM_PATH=direct python tools/r06_seg_gemm.py
(no FX_GEMM_PATH: the planner's choice)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402

PEAK = 157.3


def timeit(fn, iters=100):
    for _ in range(10):
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
    dev = "cuda"
    path = os.environ.get("FX_GEMM_PATH", "planner")
    shapes = ((102, 512, 512, "nn"), (192, 512, 512, "nn"), (256, 512, 512, "nn"), (384, 512, 512, "nn"),
              (192, 768, 512, "nn"), (192, 256, 1024, "nn"), (192, 512, 512, "nt"), (102, 512, 512, "nt"),
              (512, 513, 192, "tn"), (512, 513, 102, "tn"), (256, 257, 192, "tn"))
    if os.environ.get("SWEEP"):   # where the direct kernel stops paying: more rows, deeper K
        shapes = tuple((M, N, 512, "nn") for M in (512, 768, 1024, 1536, 2048, 4096) for N in (256, 512)) + \
            tuple((192, 512, K, "nn") for K in (1024, 2048)) + ((768, 512, 512, "nt"), (1536, 512, 512, "nt")) + \
            tuple((512, 513, K, "tn") for K in (256, 384, 512, 768, 1024, 2048)) + ((256, 257, 512, "tn"), (256, 257, 1024, "tn"))
    for M, N, K, kind in shapes:
        if kind == "nn":      # y = x W^T (Linear forward)
            a = torch.randn(M, K, device=dev)
            b = torch.randn(N, K, device=dev)
            ao, bo = fxf._rows_operand(a), fxf._rows_operand(b)
        elif kind == "nt":    # dx = dy W (Linear input gradient)
            a = torch.randn(M, K, device=dev)
            b = torch.randn(K, N, device=dev)
            ao, bo = fxf._rows_operand(a), fxf._rows_operand(b, trans=True)
        else:                 # dW = dy^T x (Linear weight gradient, K = rows)
            a = torch.randn(K, M, device=dev)
            b = torch.randn(K, N, device=dev)
            ao, bo = fxf._rows_operand(a, trans=True), fxf._rows_operand(b, trans=True)
        c = torch.empty(M, N, device=dev)
        ref = None
        if kind == "nn":
            ref = a @ b.t()
        elif kind == "nt":
            ref = a @ b
        else:
            ref = a.t() @ b

        for split in (1, 4):
            def run():
                fxf.gemm(M, N, K, ao, bo, c, N, split=split)
            us = timeit(run)
            err = (c - ref).abs().max().item() / ref.abs().max().item()
            tf = 2 * M * N * K / (us * 1e-6) / 1e12
            print(f"{path:8s} {kind} M={M:4d} N={N:4d} K={K:5d} split {split} {us:8.2f} us {tf:7.2f} TF/s  "
                  f"rel err {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
