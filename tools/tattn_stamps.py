"""Diagnostic: where one attention-over-T forward launch (tattn_fwd32_kernel, the headline shape: 2 videos,
32 queries, T = 4096, head dim 32, 8 heads; 16 chunks of 256 keys per (video, head) = 256 workgroups) spends its
time, from s_memrealtime stamps of thread 0 of every workgroup (diagnostic build: attn_t.hip with
-DTATTN_STAMPS, loaded through FACTMX_LIB).  Stamps: 0 start, 1 loads + S = q K^T done, 2 P V done and the wave
partials in LDS, 3 the chunk partial stored (issued), 4 its stores acknowledged, 5 arrival counted, 6 merge done
(the last arriver of each (video, head) only)."""
import ctypes
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fact-clip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from factmx import native as nx  # noqa: E402


def main():
    lib = nx.load()
    nvid, Lq, T, hd, nh, NL = 2, 32, 4096, 32, 8, 6
    A = hd * nh
    ld = 2 * A * NL
    q = torch.randn(nvid * Lq, A, device="cuda")
    kv = torch.randn(nvid * T, ld, device="cuda")
    o = torch.empty_like(q)
    lse = torch.empty(nvid, nh, Lq, device="cuda")
    ws = torch.empty(lib.fx_mha_t_workspace_floats(nvid, Lq, T, hd, nh), device="cuda")
    sc = ctypes.c_float(1 / math.sqrt(hd))
    vp = kv[:, A * NL:]
    fn = lib.fx_debug_tattn_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = np.zeros(1024 * 8, dtype=np.uint64)
    for it in range(8):
        nx.check(lib.fx_mha_t_fwd(nx.ptr(q), A, nx.ptr(kv), ld, nx.ptr(vp), ld, nvid, Lq, T, hd, nh, sc, nx.ptr(o), A,
                                  nx.ptr(lse), nx.ptr(ws), nx.stream()), "fwd")
        torch.cuda.synchronize()
        if it < 5:
            continue
        assert fn(buf.ctypes.data) == 0
        st = buf.reshape(1024, 8)[:256].astype(np.int64)
        t0 = st[:, 0].min()
        rel = (st - t0) / 100.0
        last = st[:, 6] > st[:, 0]
        print(f"launch: start skew {rel[:, 0].max():.2f} us; all partials acknowledged by {rel[:, 4].max():.2f} us; "
              f"last merge done {rel[last, 6].max():.2f} us ({last.sum()} mergers)")
        names = ["loads+S", "PV+LDS", "partial", "ack", "arrive"]
        for k, n in enumerate(names):
            d = rel[:, k + 1] - rel[:, k]
            print(f"  {n:8s} median {np.median(d):6.2f}  min {d.min():6.2f}  max {d.max():6.2f} us")
        d = rel[last, 6] - rel[last, 5]
        print(f"  {'merge':8s} median {np.median(d):6.2f}  min {d.min():6.2f}  max {d.max():6.2f} us")
        s0 = rel[:, 0]
        print("  start by block id (16 per (video, head)): " + " ".join(f"{s0[g * 16:(g + 1) * 16].min():.1f}-"
                                                                  f"{s0[g * 16:(g + 1) * 16].max():.1f}" for g in range(16)))
        print("  start by chunk (mean over the 16 (video, head)): " +
              " ".join(f"{s0.reshape(16, 16)[:, c].mean():.1f}" for c in range(16)))
        print(f"  arrival spread per (video, head): median "
              f"{np.median([np.ptp(rel[g * 16:(g + 1) * 16, 5]) for g in range(16)]):.2f} us")


if __name__ == "__main__":
    main()
