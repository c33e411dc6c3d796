"""Kernel-level numerics of the HIP path vs float64 references of the same ops (GPU)."""
import ctypes

import numpy as np
import pytest
import torch

from factmx import functional as fxf
from factmx import native as nx
from oracle import fact_oracle as fo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale)


def _close(a, b, rtol=2e-5, atol=2e-5, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item() if a.numel() else 0.0
    ref = b.abs().max().item() if b.numel() else 0.0
    assert err <= atol + rtol * ref, f"{what}: max err {err:.3e} (ref max {ref:.3e})"


@pytest.mark.parametrize("M,N,K", [(64, 64, 32), (4096, 256, 256), (37, 75, 53), (1, 5, 3), (300, 512, 437)])
def test_linear_fwd_bwd(M, N, K):
    x = _r(M, K, seed=1)
    w = _r(N, K, seed=2, scale=K ** -0.5)
    b = _r(N, seed=3)
    g = _r(M, N, seed=4)
    xd, wd, bd = (t.float().to(DEV).requires_grad_(True) for t in (x, w, b))
    y = fxf.linear(xd, wd, bd)
    (y * g.float().to(DEV)).sum().backward()
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr.t() + br
    (yr * g).sum().backward()
    _close(y, yr, what="y")
    _close(xd.grad, xr.grad, what="dx")
    _close(wd.grad, wr.grad, rtol=5e-5, what="dw")
    _close(bd.grad, br.grad, rtol=5e-5, what="db")


def test_linear_relu_strided_input():
    x = _r(200, 512, seed=5)
    w = _r(64, 437, seed=6, scale=0.05)
    xd = x.float().to(DEV)[:, :437].requires_grad_(False)
    y = fxf.linear(xd, w.float().to(DEV), None, relu=True)
    _close(y, torch.relu(x[:, :437] @ w.t()), what="strided relu linear")


@pytest.mark.parametrize("dil,T,nvid", [(1, 256, 1), (64, 256, 1), (512, 1100, 1), (4, 100, 3)])
def test_conv3_fwd_bwd(dil, T, nvid):
    C = 64
    x = _r(T * nvid, C, seed=7)
    w = _r(C, C, 3, seed=8, scale=0.1)
    b = _r(C, seed=9)
    g = _r(T * nvid, C, seed=10)
    xd, wd, bd = (t.float().to(DEV).requires_grad_(True) for t in (x, w, b))
    y = fxf.conv3(xd, wd, bd, dil, T)
    (y * g.float().to(DEV)).sum().backward()
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    yr = torch.cat([fo.dilated_conv3(xr[v * T:(v + 1) * T], wr, br, dil) for v in range(nvid)])
    (yr * g).sum().backward()
    _close(y, yr, what="conv y")
    _close(xd.grad, xr.grad, what="conv dx")
    _close(wd.grad, wr.grad, rtol=1e-4, what="conv dw")
    _close(bd.grad, br.grad, rtol=1e-4, what="conv db")


def test_gemm_concat_gather_and_splitk():
    T, S, Fs, H, N = 500, 17, 32, 48, 40
    seg = _r(S, Fs, seed=11)
    frame = _r(T, H, seed=12)
    seg_id = torch.sort(torch.randint(0, S, (T,), generator=torch.Generator().manual_seed(3)))[0]
    w = _r(N, Fs + H, seed=13, scale=0.1)
    ref = torch.cat([seg[seg_id], frame], 1) @ w.t()
    sd, fd, wd = seg.float().to(DEV), frame.float().to(DEV), w.float().to(DEV)
    sid = seg_id.to(torch.int32).to(DEV)
    y = torch.empty(T, N, device=DEV)
    a = fxf._rows_operand(sd)
    a.rows0 = nx.ptr(sid)
    a.ptr1, a.ld1, a.k_split = nx.ptr(fd), H, Fs
    fxf.gemm(T, N, Fs + H, a, fxf._rows_operand(wd), y, N)
    _close(y, ref, what="concat+gather")
    # split-K transposed-A product: dW = g^T x over a long frame axis
    g = _r(3000, 20, seed=14)
    x = _r(3000, 30, seed=15)
    out = torch.empty(20, 30, device=DEV)
    gd, xd = g.float().to(DEV), x.float().to(DEV)
    fxf.gemm(20, 30, 3000, fxf._rows_operand(gd, trans=True), fxf._rows_operand(xd, trans=True), out, 30, split=8)
    _close(out, g.t() @ x, rtol=1e-4, what="split-K")


def test_layernorm_fused_residual_relu():
    x, r = _r(300, 256, seed=16), _r(300, 256, seed=17)
    w, b = 1 + 0.1 * _r(256, seed=18), 0.1 * _r(256, seed=19)
    g = _r(300, 256, seed=20)
    for relu in (False, True):
        ts = [t.float().to(DEV).requires_grad_(True) for t in (x, r, w, b)]
        y = fxf.layer_norm(ts[0], ts[2], ts[3], 1e-5, residual=ts[1], relu=relu)
        (y * g.float().to(DEV)).sum().backward()
        rs = [t.clone().requires_grad_(True) for t in (x, r, w, b)]
        yr = fo.layer_norm(rs[0] + rs[1], rs[2], rs[3])
        if relu:
            yr = torch.relu(yr)
        (yr * g).sum().backward()
        _close(y, yr, what="ln y")
        for a_, b_, n in zip(ts, rs, "xrwb"):
            _close(a_.grad, b_.grad, rtol=1e-4, atol=1e-4, what=f"ln d{n}")


def test_process_feature_and_l2norm():
    x = _r(123, 512, seed=21)
    g = _r(123, 512, seed=22)
    gc = _r(123, 75, seed=23)
    xd = x.float().to(DEV).requires_grad_(True)
    out, cl = fxf.process_feature(xd, 75)
    ((out * g.float().to(DEV)).sum() + (cl * gc.float().to(DEV)).sum()).backward()
    xr = x.clone().requires_grad_(True)
    outr, clr = fo.process_feature(xr, 75)
    ((outr * g).sum() + (clr * gc).sum()).backward()
    _close(out, outr, what="pf")
    _close(xd.grad, xr.grad, what="pf dx")
    xd = x.float().to(DEV).requires_grad_(True)
    y = fxf.l2_normalize(xd)
    (y * g.float().to(DEV)).sum().backward()
    xr = x.clone().requires_grad_(True)
    yr = xr / xr.norm(dim=-1, keepdim=True).clamp_min(1e-12)
    (yr * g).sum().backward()
    _close(y, yr, what="l2n")
    _close(xd.grad, xr.grad, what="l2n dx")


@pytest.mark.parametrize("Lq,Lk,E,nh", [(32, 4096, 256, 8), (32, 32, 256, 8), (8, 200, 32, 4), (6, 6, 16, 4)])
def test_mha(Lq, Lk, E, nh):
    torch.manual_seed(0)
    mod = torch.nn.MultiheadAttention(E, nh, kdim=2 * E if Lk > 100 else None, vdim=2 * E if Lk > 100 else None,
                                      dropout=0.0).double()
    kd = 2 * E if Lk > 100 else E
    q, k, v = _r(Lq, E, seed=24), _r(Lk, kd, seed=25), _r(Lk, kd, seed=26)
    g = _r(Lq, E, seed=27)
    modd = torch.nn.MultiheadAttention(E, nh, kdim=kd, vdim=kd, dropout=0.0).to(DEV)
    modd.load_state_dict({kk: vv.float() for kk, vv in mod.state_dict().items()})
    qd, kd_, vd = (t.float().to(DEV).requires_grad_(True) for t in (q, k, v))
    y = fxf.mha(modd, qd, kd_, vd)
    (y * g.float().to(DEV)).sum().backward()
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    P = dict(mod.named_parameters())
    yr = fo.mha(P, "", qr, kr, vr, nh)
    (yr * g).sum().backward()
    _close(y, yr, what="mha y")
    _close(qd.grad, qr.grad, rtol=1e-4, what="mha dq")
    _close(kd_.grad, kr.grad, rtol=1e-4, what="mha dk")
    _close(vd.grad, vr.grad, rtol=1e-4, what="mha dv")
    for n, p in modd.named_parameters():
        _close(p.grad, P[n].grad, rtol=1e-4, atol=1e-4, what=f"mha d{n}")


@pytest.mark.parametrize("S,In,Hh,relu", [(1, 512, 256, False), (40, 512, 256, False), (300, 64, 32, False),
                                           (7, 48, 24, False), (40, 512, 256, True), (300, 64, 32, True)])
def test_gru_bidirectional(S, In, Hh, relu):
    """fxf.gru against the fp64 oracle; relu: the UpdateBlockTDU's relu(seg_update(x)) (blocks.py:432) folded
    into the recurrence kernels (forward output and backward gate) against torch.relu of the oracle."""
    mod = torch.nn.GRU(In, Hh, 1, bidirectional=True).double()
    x = _r(S, In, seed=28)
    g = _r(S, 2 * Hh, seed=29)
    modd = torch.nn.GRU(In, Hh, 1, bidirectional=True).to(DEV)
    modd.load_state_dict({k: v.float() for k, v in mod.state_dict().items()})
    xd = x.float().to(DEV).requires_grad_(True)
    y = fxf.gru(modd, xd, relu=relu)
    (y * g.float().to(DEV)).sum().backward()
    xr = x.clone().requires_grad_(True)
    P = dict(mod.named_parameters())
    yr = fo.gru(P, "", xr, 1)
    if relu:
        yr = torch.relu(yr)
        assert (yr == 0).any() and (yr > 0).any()
    (yr * g).sum().backward()
    _close(y, yr, what="gru y")
    _close(xd.grad, xr.grad, rtol=1e-4, atol=1e-4, what="gru dx")
    for n, p in modd.named_parameters():
        _close(p.grad, P[n].grad, rtol=1e-4, atol=1e-4, what=f"gru d{n}")


def test_segments_bit_exact():
    rng = np.random.default_rng(0)
    for T, C in ((1, 5), (7, 3), (4096, 75), (5000, 2)):
        lab = np.repeat(rng.integers(0, C, T), rng.integers(1, 9, T))[:T]
        x = rng.standard_normal((T, C)).astype(np.float32) * 0.01
        x[np.arange(T), lab] += 1.0
        if T > 10:
            x[3, :] = 0.5   # ties -> first max
        xd = torch.from_numpy(x).to(DEV)
        S, sid, st, en = fxf.segments_from_probs(xd, 0, C)
        pred = x.argmax(1)
        from oracle import segments as sg
        _, s_ref, e_ref = sg.run_length_segments(pred)
        assert S == len(s_ref)
        np.testing.assert_array_equal(st.cpu().numpy(), s_ref)
        np.testing.assert_array_equal(en.cpu().numpy(), e_ref)
        np.testing.assert_array_equal(sid.cpu().numpy(), sg.segment_ids_from_bounds(s_ref, e_ref, T))


def test_library_reports_errors():
    lib = nx.load()
    st = lib.fx_layernorm_fwd(None, 0, None, 0, None, None, 1e-5, 4, 4096, 0, None, 0, None, 0, None, None)
    assert st != 0 and b"cols" in lib.fx_last_error()


@pytest.mark.parametrize("M,K,N", [(300, 437, 512), (4096, 437, 512), (64, 70, 33)])
def test_linear_padded_k_on_wider_input(M, K, N):
    """LinearPadKFn (K not a multiple of 64, input a column slice of a wider tensor) vs float64."""
    Kw = (K + 63) // 64 * 64 + 64
    xw = _r(M, Kw, seed=40)
    w = _r(N, K, seed=41, scale=K ** -0.5)
    b = _r(N, seed=42)
    g = _r(M, N, seed=43)
    xwd = xw.float().to(DEV).requires_grad_(True)
    wd, bd = w.float().to(DEV).requires_grad_(True), b.float().to(DEV).requires_grad_(True)
    y = fxf.linear_any_k(xwd[:, :K], wd, bd)
    (y * g.float().to(DEV)).sum().backward()
    xr = xw.clone().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    yr = xr[:, :K] @ wr.t() + br
    (yr * g).sum().backward()
    _close(y, yr, what="y")
    _close(xwd.grad, xr.grad, rtol=1e-4, atol=1e-4, what="dx")
    _close(wd.grad, wr.grad, rtol=1e-4, atol=1e-4, what="dw")
    _close(bd.grad, br.grad, rtol=1e-4, atol=1e-4, what="db")


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("T,nvid,nl", [(1000, 2, 10), (4096, 1, 3), (37, 3, 4), ((1000, 777, 1301), 3, 10),
                                       ((64, 5, 200), 3, 4)])
def test_mstcn_fused_layers_match_fp64(T, nvid, nl, fused, monkeypatch):
    """F = 256, both MS-TCN paths: the two-GEMM layers and (fx_mstcn_params.fused_layers) the fused
    layer kernel (mstcn_fused.hip) forward + fused dX chain backward: output, input gradient and every
    weight gradient vs the float64 MS-TCN restatement (odd row counts, dilations up to 2^(nl-1),
    several videos: no leakage across video edges).  A tuple T is a ragged batch (row offsets through
    the conv GEMMs and the fused layer's tap gather, up to 16 videos; the deferred weight gradients in
    one launch per weight kind, the ragged frame lookup in the GEMM's B loader over K = rows rounded up
    to the 64-deep stage)."""
    from factmx.dp import FlatGradReducer
    from factmx.models.basic import MSTCN
    monkeypatch.setattr(fxf, "MSTCN_FUSED_LAYERS", 2 if fused == "1" else 0)   # 2: the fused kernel at any size
    torch.manual_seed(0)
    mod = MSTCN(96, 256, 40, nl, dropout=0.0, ln=False, in_map=True).to(DEV).train()
    Ts = list(T) if isinstance(T, tuple) else [T] * nvid
    off = [0]
    for t_ in Ts:
        off.append(off[-1] + t_)
    rows = off[-1]
    x = _r(rows, 96, seed=11)
    g = _r(rows, 40, seed=12)
    xd = x.float().to(DEV).requires_grad_(True)
    if isinstance(T, tuple):
        FlatGradReducer(mod.parameters())        # uniformly strided gradients: the deferred batched dW path
        y = fxf.mstcn(mod, xd, T=0, nvid=nvid, seq_off=off)
    else:
        y = fxf.mstcn(mod, xd, T=T, nvid=nvid)
    saved = y.grad_fn.saved_tensors[1].detach().double().cpu()   # (freed by the backward)
    (y * g.float().to(DEV)).sum().backward()
    # the float64 restatement takes the GPU's own ReLU decisions (z > 0 of the saved activations):
    # a pre-activation within ~1e-6 of 0 may land on the other side in fp32 (either summation order
    # is valid), which would move single dZ entries -- whole conv-weight-gradient rows -- by O(1)
    # (the GRU kink of tests/helpers.GruKinks); with the same gates everything agrees at fp32 noise
    n = -(-rows // 64) * 64 * 256         # per-layer slot: rows rounded up to the 64-deep GEMM stage
    gates = [(saved[(nl + 1 + i) * n:(nl + 1 + i) * n + rows * 256].view(rows, 256) > 0).double() for i in range(nl)]
    P = {n_: t.detach().double().cpu().requires_grad_(True) for n_, t in mod.named_parameters()}
    xr = x.clone().requires_grad_(True)
    outs = []
    for v in range(nvid):
        sl = slice(off[v], off[v + 1])
        h = fo.linear(xr[sl], P["conv_1x1.weight"], P["conv_1x1.bias"])
        for i in range(nl):
            q = f"layers.{i}."
            z = fo.dilated_conv3(h, P[q + "conv_dilated.weight"], P[q + "conv_dilated.bias"], 2 ** i) * gates[i][sl]
            h = h + fo.linear(z, P[q + "conv_1x1.weight"], P[q + "conv_1x1.bias"])
        outs.append(fo.linear(h, P["conv_out.weight"], P["conv_out.bias"]))
    yr = torch.cat(outs, 0)
    (yr * g).sum().backward()
    _close(y, yr, rtol=1e-4, atol=1e-4, what="y")
    _close(xd.grad, xr.grad, rtol=1e-4, atol=1e-4, what="dx")
    for n_, t in mod.named_parameters():
        _close(t.grad, P[n_].grad, rtol=2e-4, atol=2e-4, what=f"d{n_}")
