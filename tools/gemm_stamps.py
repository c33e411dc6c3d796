"""Where does a GEMM launch spend its time?  (diagnostic; needs `make -C fact-clip_amd/csrc stamps`)

FACTMX_LIB=fact-clip_amd/factmx/_lib/libfactmx_stamps.so python tools/gemm_stamps.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
os.environ.setdefault("FACTMX_LIB", os.path.join(ROOT, "fact-clip_amd", "factmx", "_lib", "libfactmx_stamps.so"))

import ctypes  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402
from factmx import native as nx  # noqa: E402


def run(M, N, K, a, b, c, ldc, **kw):
    lib = nx.load()
    tiles = ((N + 63) // 64) * ((M + 63) // 64)
    st = torch.zeros(tiles * 2 * 10, dtype=torch.int64, device="cuda")
    d = nx.GemmDesc()
    d.M, d.N, d.K, d.batch = M, N, K, 1
    d.a, d.b = a, b
    d.c, d.ldc = nx.ptr(c), ldc
    d.alpha = 1.0
    d.bias = nx.ptr(kw.get("bias"))
    d.relu = kw.get("relu", 0)
    d.split_k = 1
    d.dbg_stamps = nx.ptr(st)
    for _ in range(20):
        nx.check(lib.fx_gemm(ctypes.byref(d), nx.stream()), "gemm")
    torch.cuda.synchronize()
    s = st.cpu().numpy().reshape(tiles, 2, 5, 2)   # block, wave group, slot, (memtime, realtime)
    return s


def report(name, s):
    mt = s[:, 0, :, 0].astype(np.float64)
    rt = s[:, 0, :, 1].astype(np.float64)
    loop = mt[:, 2] - mt[:, 0]     # prologue + k loop (slot 1 is not stamped)
    epi = mt[:, 3] - mt[:, 2]
    span = (rt[:, 3].max() - rt[:, 0].min()) * 10.0   # 100 MHz -> ns
    start_spread = (rt[:, 0].max() - rt[:, 0].min()) * 10.0
    clk = (mt[:, 3] - mt[:, 0]) / ((rt[:, 3] - rt[:, 0]) * 10.0)   # cycles per ns
    print(f"{name}: blocks {len(mt)} span {span/1e3:.2f} us, start spread {start_spread/1e3:.2f} us, clock {np.median(clk):.2f} GHz")
    for lab, v in (("k-loop", loop), ("epilogue", epi)):
        print(f"   {lab:9s} cycles median {np.median(v):9.0f}  min {v.min():9.0f}  max {v.max():9.0f}")


def main():
    dev = "cuda"
    T, F = 4096, 256
    x = torch.randn(T, F, device=dev)
    w = torch.randn(F, F, 3, device=dev) * 0.05
    wf = w.permute(0, 2, 1).reshape(F, 3 * F).contiguous()
    y = torch.empty(T, F, device=dev)
    b = torch.randn(F, device=dev)
    s = run(T, F, 3 * F, fxf._conv_operand(x, F, 8, 1, T, False), fxf._rows_operand(wf), y, F, bias=b, relu=1)
    report("conv fwd M=4096 N=256 K=768", s)
    w1 = torch.randn(F, F, device=dev)
    s = run(T, F, F, fxf._rows_operand(x), fxf._rows_operand(w1), y, F)
    report("1x1 fwd  M=4096 N=256 K=256", s)
    xin = torch.randn(T, 2048, device=dev)
    win = torch.randn(F, 2048, device=dev)
    s = run(T, F, 2048, fxf._rows_operand(xin), fxf._rows_operand(win), y, F)
    report("in-map   M=4096 N=256 K=2048", s)


if __name__ == "__main__":
    main()
