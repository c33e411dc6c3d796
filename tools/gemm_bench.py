"""Micro-benchmark of the f32 MFMA GEMM on the FACT frame-branch shapes (diagnostic).

python tools/gemm_bench.py   -> one line per shape: avg us, TFLOP/s, fraction of 157.3 TF
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402

PEAK = 157.3


def timeit(fn, iters=50):
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
    dev = "cuda"
    T, F, H = 4096, 256, 512
    rows = int(os.environ.get("ROWS", T))
    x = torch.randn(rows, F, device=dev)
    w = torch.randn(F, F, 3, device=dev) * 0.05
    wf = w.permute(0, 2, 1).reshape(F, 3 * F).contiguous()
    wb = w.permute(1, 2, 0).reshape(F, 3 * F).contiguous()
    y = torch.empty(rows, F, device=dev)
    dw = torch.zeros(F, F, 3, device=dev)
    db = torch.zeros(F, device=dev)
    w1 = torch.randn(F, F, device=dev) * 0.05
    xin = torch.randn(rows, 2048, device=dev)
    win = torch.randn(F, 2048, device=dev) * 0.02
    tok = torch.randn(32, F, device=dev)
    wt = torch.randn(2 * F, F, device=dev)
    cases = []

    def conv_fwd():
        fxf.gemm(rows, F, 3 * F, fxf._conv_operand(x, F, 8, 1, T, False), fxf._rows_operand(wf), y, F, relu=1)
    cases.append(("conv fwd  M=%d N=256 K=768" % rows, conv_fwd, 2 * rows * F * 3 * F))

    def conv_dx():
        fxf.gemm(rows, F, 3 * F, fxf._conv_operand(x, F, 8, -1, T, False), fxf._rows_operand(wb), y, F, resid=x)
    cases.append(("conv dX   M=%d N=256 K=768" % rows, conv_dx, 2 * rows * F * 3 * F))

    def conv_dw():
        b = fxf._conv_operand(x, F, 8, 1, T, True)
        b.ones_col = 3 * F + 1
        fxf.gemm(F, 3 * F + 1, rows, fxf._rows_operand(y, trans=True), b, dw, 3 * F, c_tap_cin=F, split=7, beta=1.0,
                 c_last=db)
    cases.append(("conv dW   M=256 N=769 K=%d split7" % rows, conv_dw, 2 * rows * F * (3 * F + 1)))

    def pw_fwd():
        fxf.gemm(rows, F, F, fxf._rows_operand(x), fxf._rows_operand(w1), y, F, resid=x)
    cases.append(("1x1 fwd   M=%d N=256 K=256" % rows, pw_fwd, 2 * rows * F * F))

    def pw_dx():
        fxf.gemm(rows, F, F, fxf._rows_operand(x), fxf._rows_operand(w1, trans=True), y, F, gate=x)
    cases.append(("1x1 dX    M=%d N=256 K=256 (B cols)" % rows, pw_dx, 2 * rows * F * F))

    def in_fwd():
        fxf.gemm(rows, F, 2048, fxf._rows_operand(xin), fxf._rows_operand(win), y, F)
    cases.append(("in-map    M=%d N=256 K=2048" % rows, in_fwd, 2 * rows * F * 2048))

    out_t = torch.empty(32, 2 * F, device=dev)

    def tok_fwd():
        fxf.gemm(32, 2 * F, F, fxf._rows_operand(tok), fxf._rows_operand(wt), out_t, 2 * F)
    cases.append(("token     M=32 N=512 K=256", tok_fwd, 2 * 32 * 2 * F * F))

    only = os.environ.get("CASE")
    precs = os.environ.get("PREC", "fp32").split(",")
    for name, fn, fl in cases:
        if only and not name.startswith(only):
            continue
        for prec in precs:
            with fxf.gemm_precision(prec):
                us = timeit(fn)
            tf = fl / (us * 1e-6) / 1e12
            print(f"{name:40s} {prec:6s} {us:8.2f} us  {tf:7.2f} TF/s  {tf / PEAK:6.3f} of f32 peak", flush=True)


if __name__ == "__main__":
    main()
