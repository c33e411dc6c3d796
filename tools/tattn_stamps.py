"""Diagnostic: per-phase cycle stamps of the fused attention-over-T forward (libfactmx_stamps.so).
FACTMX_LIB=fact-clip_amd/factmx/_lib/libfactmx_stamps.so python tools/tattn_stamps.py"""
import ctypes
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("FACTMX_LIB", os.path.join(ROOT, "fact-clip_amd", "factmx", "_lib", "libfactmx_stamps.so"))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from factmx import native as nx  # noqa: E402

lib = nx.load()
lib.fx_dbg_tattn_stamps.argtypes = [ctypes.c_void_p]
for T in (4096, 16384):
    nvid, Lq, hd, nh, NL = 2, 32, 32, 8, 6
    A = hd * nh
    ld = 2 * A * NL
    q = torch.randn(nvid * Lq, A, device="cuda")
    kv = torch.randn(nvid * T, ld, device="cuda")
    o = torch.empty_like(q)
    lse = torch.empty(nvid, nh, Lq, device="cuda")
    ws = torch.empty(lib.fx_mha_t_workspace_floats(nvid, Lq, T, hd, nh), device="cuda")
    st = torch.zeros(4096 * 8, dtype=torch.int64, device="cuda")
    sc = ctypes.c_float(1 / math.sqrt(hd))

    def fwd():
        nx.check(lib.fx_mha_t_fwd(nx.ptr(q), A, nx.ptr(kv), ld, nx.ptr(kv[:, A * NL:]), ld, nvid, Lq, T, hd, nh, sc,
                                  nx.ptr(o), A, nx.ptr(lse), nx.ptr(ws), nx.stream()), "fwd")
    lib.fx_dbg_tattn_stamps(None)
    for _ in range(3):
        fwd()
    torch.cuda.synchronize()
    lib.fx_dbg_tattn_stamps(ctypes.c_void_p(st.data_ptr()))
    fwd()
    torch.cuda.synchronize()
    lib.fx_dbg_tattn_stamps(None)
    s = st.view(-1, 8).cpu().numpy()
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    print(f"T={T}: {len(s)} workgroups")
    names = ["stage", "S", "softmax", "PV+store"]
    for i, n in enumerate(names):
        d = s[:, i + 1] - s[:, i]
        print(f"  {n:9s} mean {d.mean():8.0f}  p50 {np.median(d):8.0f}  max {d.max():8.0f} cycles")
