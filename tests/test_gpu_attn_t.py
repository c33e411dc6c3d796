"""Fused multi-head attention over T frames (fx_mha_t_fwd / fx_mha_t_bwd, attn_t.hip) against a
float64 torch restatement of nn.MultiheadAttention's core (basic.py:508-516): o, log-sum-exp and
the dq / dk / dv gradients, on the benchmark shape (2 videos x 32 tokens x 4096 frames, 8 heads of
32, K and V as column ranges of one packed (T, 2 A L) projection like fx_decoder), the Breakfast
shape (60 tokens, head dim 64) and ragged sizes (T not a multiple of the chunk, 3 videos, fewer
queries than a 32-row tile)."""
import ctypes
import math

import pytest
import torch

from factmx import native as nx

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, nvid, Lq, T, hd, nh, scale, dout):
    q, k, v = (t.detach().double().cpu().requires_grad_(True) for t in (q, k, v))
    outs, lses = [], []
    for b in range(nvid):
        qb, kb, vb = q[b * Lq:(b + 1) * Lq], k[b * T:(b + 1) * T], v[b * T:(b + 1) * T]
        ob, lb = [], []
        for h in range(nh):
            sl = slice(h * hd, (h + 1) * hd)
            s = qb[:, sl] @ kb[:, sl].t() * scale
            lb.append(torch.logsumexp(s, -1))
            ob.append(torch.softmax(s, -1) @ vb[:, sl])
        outs.append(torch.cat(ob, 1))
        lses.append(torch.stack(lb, 0))
    o = torch.cat(outs, 0)
    (o * dout.double().cpu()).sum().backward()
    return o.detach(), torch.stack(lses, 0).detach(), q.grad, k.grad, v.grad


# head dim 32 with <= 32 queries runs the register-resident kernels (256- or 128-key chunks merged inside
# the launch by the last workgroup of each (video, head); one chunk: no merge; > 16 chunks (T = 5000): the
# merge launch); the others the LDS-staged ones
@pytest.mark.parametrize("nvid,Lq,T,hd,nh", [(2, 32, 4096, 32, 8), (1, 60, 512, 64, 8), (3, 8, 200, 16, 2),
                                             (2, 64, 1000, 64, 4), (3, 20, 1000, 32, 4), (1, 32, 100, 32, 8),
                                             (2, 32, 300, 32, 8), (16, 32, 512, 32, 8), (2, 32, 5000, 32, 8)])
def test_mha_over_t_matches_fp64(nvid, Lq, T, hd, nh):
    lib = nx.load()
    A = hd * nh
    g = torch.Generator().manual_seed(7)
    q = torch.randn(nvid * Lq, A, generator=g)
    kv = torch.randn(nvid * T, 3 * A, generator=g)          # packed [k | spare | v] rows, ld 3A
    dout = torch.randn(nvid * Lq, A, generator=g)
    k, v = kv[:, :A], kv[:, 2 * A:]
    scale = 1.0 / math.sqrt(hd)
    qd, kvd, doutd = q.to(DEV), kv.to(DEV), dout.to(DEV)
    o = torch.empty(nvid * Lq, A, device=DEV)
    lse = torch.empty(nvid, nh, Lq, device=DEV)
    ws = torch.empty(max(lib.fx_mha_t_workspace_floats(nvid, Lq, T, hd, nh), 1), device=DEV)
    nx.check(lib.fx_mha_t_fwd(nx.ptr(qd), A, nx.ptr(kvd), 3 * A, nx.ptr(kvd[:, 2 * A:]), 3 * A, nvid, Lq, T, hd, nh,
                              ctypes.c_float(scale), nx.ptr(o), A, nx.ptr(lse), nx.ptr(ws), nx.stream()), "fx_mha_t_fwd")
    dq = torch.empty_like(qd)
    dkv = torch.full_like(kvd, 7.0)                          # the spare columns must stay untouched
    nx.check(lib.fx_mha_t_bwd(nx.ptr(qd), A, nx.ptr(kvd), 3 * A, nx.ptr(kvd[:, 2 * A:]), 3 * A, nx.ptr(o), A,
                              nx.ptr(doutd), A, nx.ptr(lse), nvid, Lq, T, hd, nh, ctypes.c_float(scale), nx.ptr(dq), A,
                              nx.ptr(dkv), 3 * A, nx.ptr(dkv[:, 2 * A:]), 3 * A, nx.ptr(ws), nx.stream()),
             "fx_mha_t_bwd")
    torch.cuda.synchronize()
    o_r, lse_r, dq_r, dk_r, dv_r = _ref(q, k, v, nvid, Lq, T, hd, nh, scale, dout)

    def close(got, ref, what, tol=2e-5):
        err = (got.double().cpu() - ref).abs().max().item()
        assert err <= tol * max(1.0, ref.abs().max().item()), (what, err)
    close(o, o_r, "o")
    close(lse, lse_r, "lse")
    close(dq, dq_r, "dq")
    close(dkv[:, :A], dk_r, "dk")
    close(dkv[:, 2 * A:], dv_r, "dv")
    assert torch.all(dkv[:, A:2 * A] == 7.0)
    # the in-launch merge re-arms its arrival counters: repeated launches are bitwise identical
    o2, lse2, dq2, dkv2 = torch.empty_like(o), torch.empty_like(lse), torch.empty_like(dq), dkv.clone()
    for _ in range(2):
        nx.check(lib.fx_mha_t_fwd(nx.ptr(qd), A, nx.ptr(kvd), 3 * A, nx.ptr(kvd[:, 2 * A:]), 3 * A, nvid, Lq, T, hd,
                                  nh, ctypes.c_float(scale), nx.ptr(o2), A, nx.ptr(lse2), nx.ptr(ws), nx.stream()),
                 "fx_mha_t_fwd")
        nx.check(lib.fx_mha_t_bwd(nx.ptr(qd), A, nx.ptr(kvd), 3 * A, nx.ptr(kvd[:, 2 * A:]), 3 * A, nx.ptr(o2), A,
                                  nx.ptr(doutd), A, nx.ptr(lse2), nvid, Lq, T, hd, nh, ctypes.c_float(scale),
                                  nx.ptr(dq2), A, nx.ptr(dkv2), 3 * A, nx.ptr(dkv2[:, 2 * A:]), 3 * A, nx.ptr(ws),
                                  nx.stream()), "fx_mha_t_bwd")
    torch.cuda.synchronize()
    assert torch.equal(o2, o) and torch.equal(lse2, lse) and torch.equal(dq2, dq) and torch.equal(dkv2, dkv)
