"""Diagnostic: f32 GEMM time by operand kind at the batched weight-gradient shape (M=256, N=768,
K=8192 rows, batch 10): row-major (k contiguous) vs column-major (k strided) A / B images.

python tools/cols_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402
from factmx import native as nx  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def op(t, trans, bs):
    o = fxf._rows_operand(t, trans=trans)
    o.batch_stride = bs
    return o


def main():
    M, N, K, B = 256, 768, 8192, int(os.environ.get("NB", 10))
    dev = "cuda"
    a_cm = torch.randn(B * K, M, device=dev)     # (k, m) per batch: column-major A (dZ rows)
    a_rm = torch.randn(B * M, K, device=dev)
    b_cm = torch.randn(B * K, N, device=dev)
    b_rm = torch.randn(B * N, K, device=dev)
    c = torch.zeros(B * M, N, device=dev)
    fl = 2.0 * M * N * K * B
    cases = {
        "A cols, B cols": (op(a_cm, True, K * M), op(b_cm, True, K * N)),
        "A rows, B rows": (op(a_rm, False, M * K), op(b_rm, False, N * K)),
        "A cols, B rows": (op(a_cm, True, K * M), op(b_rm, False, N * K)),
        "A rows, B cols": (op(a_rm, False, M * K), op(b_cm, True, K * N)),
    }
    for name, (a, b) in cases.items():
        us = timeit(lambda: fxf.gemm(M, N, K, a, b, c, N, batch=B, c_bs=M * N))
        print(f"{name}: {us:8.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
    # the conv dW operand (B = shifted taps of h, column-major) at the same size
    h = torch.randn(B * K, 256, device=dev)
    bo = fxf._conv_operand(h, 256, 1, 1, 4096, True)
    bo.batch_stride = K * 256
    us = timeit(lambda: fxf.gemm(M, N, K, op(a_cm, True, K * M), bo, c, N, batch=B, c_bs=M * N, c_tap_cin=256))
    print(f"A cols, B cols_conv: {us:8.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)
    # split 8 (the deferred weight-gradient launches): 10 x 8 = 80 z-planes (plane-per-XCD mapping)
    for name, (a, b) in (("A cols, B cols", cases["A cols, B cols"]), ("A cols, B cols_conv", (op(a_cm, True, K * M), bo))):
        tap = 256 if b is bo else 0
        us = timeit(lambda: fxf.gemm(M, N, K, a, b, c, N, batch=B, c_bs=M * N, c_tap_cin=tap, split=8))
        print(f"{name} split 8: {us:8.1f} us  {fl / us / 1e6:6.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
