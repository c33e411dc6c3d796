"""Diagnostic: time fx_mha_t_fwd / fx_mha_t_bwd (fused multi-head attention over T) alone, HIP events,
K/V packed like fx_decoder's projection (row stride 2 A L).  python tools/tattn_bench.py [T ...]"""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fact-clip_amd"))
import torch  # noqa: E402

from factmx import native as nx  # noqa: E402

lib = nx.load()


def run(nvid, Lq, T, hd, nh, NL=6, it=50):
    A = hd * nh
    ld = 2 * A * NL
    q = torch.randn(nvid * Lq, A, device="cuda")
    kv = torch.randn(nvid * T, ld, device="cuda")
    dout = torch.randn_like(q)
    o = torch.empty_like(q)
    lse = torch.empty(nvid, nh, Lq, device="cuda")
    ws = torch.empty(lib.fx_mha_t_workspace_floats(nvid, Lq, T, hd, nh), device="cuda")
    dq, dkv = torch.empty_like(q), torch.empty_like(kv)
    sc = ctypes.c_float(1 / math.sqrt(hd))
    vp = kv[:, A * NL:]

    def fwd():
        nx.check(lib.fx_mha_t_fwd(nx.ptr(q), A, nx.ptr(kv), ld, nx.ptr(vp), ld, nvid, Lq, T, hd, nh, sc, nx.ptr(o), A,
                                  nx.ptr(lse), nx.ptr(ws), nx.stream()), "fwd")

    def bwd():
        nx.check(lib.fx_mha_t_bwd(nx.ptr(q), A, nx.ptr(kv), ld, nx.ptr(vp), ld, nx.ptr(o), A, nx.ptr(dout), A,
                                  nx.ptr(lse), nvid, Lq, T, hd, nh, sc, nx.ptr(dq), A, nx.ptr(dkv), ld,
                                  nx.ptr(dkv[:, A * NL:]), ld, nx.ptr(ws), nx.stream()), "bwd")
    res = []
    for f, name in ((fwd, "fwd"), (bwd, "bwd")):
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(it):
            f()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / it * 1e3
        by = nvid * T * 2 * A * 4 * (1 if name == "fwd" else 2)
        res.append(f"{name} {us:6.1f} us ({by / us / 1e3:5.0f} GB/s)")
    print(f"nvid {nvid} Lq {Lq} T {T:6d} hd {hd} h {nh}: " + "   ".join(res), flush=True)


if __name__ == "__main__":
    Ts = [int(x) for x in sys.argv[1:]] or [512, 1024, 4096, 16384]
    for T in Ts:
        run(2, 32, T, 32, 8)
    run(1, 60, 512, 64, 8)
