"""Training dropout inside the fused kernels (GPU): the counter-based mask of fx_dropout, the
MS-TCN 1x1 branch (GEMM epilogue forward, regenerated mask in backward), attention-probability
dropout (fx_mha_core) and the X2Y concat dropout, each against a float64 torch restatement that
applies the SAME mask (tests/helpers.drop_mask, the formula include/factmx.h documents):
  * the kernel's mask equals the documented formula element for element; keep rate ~ 1 - p;
  * p > 0 in eval mode, and p = 0 in training, are bitwise the no-dropout path;
  * forward and backward use the same mask (gradients match the masked fp64 reference);
  * a FACT_CLIP train step with Bi.dropout 0.2 (havid_view0_lh_pt_holdout.yaml:50) runs and is
    reproducible under torch.manual_seed.
Reference sites: basic.py:158-160 (MS-TCN), 382 (X2Y concat), MultiheadAttention(dropout=...)
at basic.py:402, 464-465."""
import math

import numpy as np
import pytest
import torch

from helpers import drop_mask, drop_subseed
from factmx import functional as fxf
from oracle import fact_oracle as fo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64) * scale


def _close(a, b, rtol=2e-5, atol=2e-5, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item()
    assert err <= atol + rtol * ref, f"{what}: max err {err:.3e} (ref max {ref:.3e})"


def _mask(seed, shape, p, idx_ld=None, col0=0):
    rows, cols = shape
    idx_ld = cols if idx_ld is None else idx_ld
    idx = np.arange(rows, dtype=np.int64)[:, None] * idx_ld + col0 + np.arange(cols, dtype=np.int64)[None, :]
    return torch.from_numpy(drop_mask(seed, idx, p).astype(np.float64))


@pytest.fixture
def fixed_seeds(monkeypatch):
    """Make every dropout site's seed a known sequence (the kernels' masks become computable)."""
    seq = iter(range(1000, 100000, 7919))
    got = []

    def nxt():
        s = next(seq) * 0x9E3779B1 % 2 ** 62
        got.append(s)
        return s
    monkeypatch.setattr(fxf, "dropout_seed", nxt)
    return got


@pytest.mark.parametrize("p", [0.2, 0.5])
def test_mask_matches_documented_formula_and_keep_rate(p):
    x = torch.randn(513, 777, device=DEV)
    seed = 0x1234567890ABCDEF
    y = fxf.dropout(x, p, seed)
    keep = _mask(seed, x.shape, p).bool()
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    expect = torch.where(keep.to(DEV), x * float(scale), torch.zeros((), device=DEV))
    assert torch.equal(y, expect)
    rate = keep.double().mean().item()
    assert abs(rate - (1 - p)) < 5 * math.sqrt(p * (1 - p) / keep.numel())
    assert torch.equal(fxf.dropout(x, 0.0, seed), x)


def _mstcn_ref(P, x, nlayers, in_map, seed, p):
    """fo.mstcn with the kernels' dropout on every layer's 1x1 branch (basic.py:158-160)."""
    h = fo.linear(x, P["conv_1x1.weight"], P["conv_1x1.bias"]) if in_map else x
    scale = 1.0 / (1.0 - float(np.float32(p)))
    for i in range(nlayers):
        q = f"layers.{i}."
        z = torch.relu(fo.dilated_conv3(h, P[q + "conv_dilated.weight"], P[q + "conv_dilated.bias"], 2 ** i))
        u = fo.linear(z, P[q + "conv_1x1.weight"], P[q + "conv_1x1.bias"])
        h = h + u * _mask(drop_subseed(seed, i), u.shape, p) * scale
    return fo.linear(h, P["conv_out.weight"], P["conv_out.bias"])


@pytest.mark.parametrize("T,F,nl,p", [(512, 64, 4, 0.2), (1000, 256, 3, 0.5)])
def test_mstcn_dropout_matches_masked_reference(T, F, nl, p, fixed_seeds):
    from factmx.models.basic import MSTCN
    torch.manual_seed(0)
    mod = MSTCN(48, F, 24, nl, dropout=p, ln=False, in_map=True).to(DEV).train()
    x = _r(T, 48, seed=1)
    g = _r(T, 24, seed=2)
    xd = x.float().to(DEV).requires_grad_(True)
    y = mod(xd.unsqueeze(1))[:, 0]
    (y * g.float().to(DEV)).sum().backward()
    seed = fixed_seeds[-1]
    P = {n: t.detach().double().cpu().requires_grad_(True) for n, t in mod.named_parameters()}
    xr = x.clone().requires_grad_(True)
    yr = _mstcn_ref(P, xr, nl, True, seed, p)
    (yr * g).sum().backward()
    _close(y, yr, rtol=1e-4, atol=1e-4, what="y")
    _close(xd.grad, xr.grad, rtol=1e-4, atol=1e-4, what="dx")
    for n, t in mod.named_parameters():
        _close(t.grad, P[n].grad, rtol=2e-4, atol=2e-4, what=f"d{n}")
    # eval mode: bitwise the no-dropout path; p = 0 in training likewise
    mod.eval()
    with torch.no_grad():
        ye = mod(xd.unsqueeze(1))
        for lyr in mod.layers:
            lyr.dropout.p = 0.0
        mod.dropout_rate = 0.0
        mod.train()
        y0 = mod(xd.unsqueeze(1))
    assert torch.equal(ye, y0)


def _mha_ref(P, q_in, k_in, v_in, nhead, seed, p):
    """fo.mha with the kernels' dropout on the attention probabilities, index (h Lq + i) Lk + j."""
    E = q_in.shape[-1]
    hd = E // nhead
    bi = P["in_proj_bias"]
    if "in_proj_weight" in P:
        W = P["in_proj_weight"]
        wq, wk, wv = W[:E], W[E:2 * E], W[2 * E:]
    else:
        wq, wk, wv = P["q_proj_weight"], P["k_proj_weight"], P["v_proj_weight"]
    q, k, v = fo.linear(q_in, wq, bi[:E]), fo.linear(k_in, wk, bi[E:2 * E]), fo.linear(v_in, wv, bi[2 * E:])
    L, S = q.shape[0], k.shape[0]
    qh = q.reshape(L, nhead, hd).transpose(0, 1)
    kh = k.reshape(S, nhead, hd).transpose(0, 1)
    vh = v.reshape(S, nhead, hd).transpose(0, 1)
    att = fo.softmax(qh @ kh.transpose(1, 2) / math.sqrt(hd))
    m = _mask(seed, (nhead * L, S), p).reshape(nhead, L, S)
    att = att * m / (1.0 - float(np.float32(p)))
    o = (att @ vh).transpose(0, 1).reshape(L, E)
    return fo.linear(o, P["out_proj.weight"], P["out_proj.bias"])


@pytest.mark.parametrize("Lq,Lk,E,nh", [(32, 1000, 64, 8), (32, 32, 256, 8)])
def test_attention_dropout_matches_masked_reference(Lq, Lk, E, nh, fixed_seeds):
    p = 0.2
    torch.manual_seed(0)
    kd = 2 * E if Lk > 100 else E
    mod = torch.nn.MultiheadAttention(E, nh, kdim=kd, vdim=kd, dropout=p).to(DEV).train()
    q, k, v = _r(Lq, E, seed=24), _r(Lk, kd, seed=25), _r(Lk, kd, seed=26)
    g = _r(Lq, E, seed=27)
    qd, kd_, vd = (t.float().to(DEV).requires_grad_(True) for t in (q, k, v))
    y = fxf.mha(mod, qd, kd_, vd)
    (y * g.float().to(DEV)).sum().backward()
    seed = fixed_seeds[-1]
    P = {n: t.detach().double().cpu().requires_grad_(True) for n, t in mod.named_parameters()}
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    yr = _mha_ref(P, qr, kr, vr, nh, seed, p)
    (yr * g).sum().backward()
    _close(y, yr, what="y")
    _close(qd.grad, qr.grad, rtol=1e-4, what="dq")
    _close(kd_.grad, kr.grad, rtol=1e-4, what="dk")
    _close(vd.grad, vr.grad, rtol=1e-4, what="dv")
    for n, t in mod.named_parameters():
        _close(t.grad, P[n].grad, rtol=1e-4, atol=1e-4, what=f"d{n}")


def test_x2y_concat_dropout_matches_masked_reference(fixed_seeds):
    from factmx.models.basic import X2Y_map
    p = 0.2
    torch.manual_seed(0)
    mod = X2Y_map(64, 48, 40, 64, dropout=p, kq_pos=True).to(DEV).train()
    X, Y = _r(300, 64, seed=3), _r(20, 48, seed=4)
    Xp, Yp = _r(300, 64, seed=5, scale=0.1), _r(20, 48, seed=6, scale=0.1)
    g = _r(20, 40, seed=7)
    Xd, Yd = (t.float().to(DEV).requires_grad_(True) for t in (X, Y))
    out = mod(Xd.unsqueeze(1), Yd.unsqueeze(1), X_pos=Xp.float().to(DEV).unsqueeze(1),
              Y_pos=Yp.float().to(DEV).unsqueeze(1))[:, 0]
    (out * g.float().to(DEV)).sum().backward()
    seed = fixed_seeds[-1]
    P = {n: t.detach().double().cpu().requires_grad_(True) for n, t in mod.named_parameters()}
    Xr, Yr = (t.clone().requires_grad_(True) for t in (X, Y))
    xk = fo.linear(fo.add_pos(Xr, Xp), P["X_K.weight"], P["X_K.bias"])
    xv = fo.linear(Xr, P["X_V.weight"], P["X_V.bias"])
    yq = fo.linear(fo.add_pos(Yr, Yp), P["Y_Q.weight"], P["Y_Q.bias"])
    attn = fo.softmax(yq @ xk.t() / math.sqrt(64), -1)
    cat = torch.cat([Yr, attn @ xv], -1)
    cat = cat * _mask(seed, cat.shape, p) / (1.0 - float(np.float32(p)))
    ref = fo.linear(cat, P["Y_W.weight"], P["Y_W.bias"])
    (ref * g).sum().backward()
    _close(out, ref, what="out")
    _close(Xd.grad, Xr.grad, rtol=1e-4, what="dX")
    _close(Yd.grad, Yr.grad, rtol=1e-4, what="dY")
    for n, t in mod.named_parameters():
        _close(t.grad, P[n].grad, rtol=1e-4, atol=1e-4, what=f"d{n}")


def test_fact_clip_trains_with_havid_dropout():
    """Bi.dropout 0.2 as havid_view0_lh_pt_holdout.yaml:50 (inherited by Bu / BU): a train step runs,
    the loss is finite, and it is reproducible under torch.manual_seed (and differs across seeds)."""
    from helpers import load_fixture, tiny_meta, cfg_from_meta, tiny_inputs
    import paramgen as pg
    from factmx.models.blocks import FACT_CLIP
    from factmx.models.loss import MatchCriterion
    fx = load_fixture("tiny_clip")
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    for sec in (cfg.Bi, cfg.Bu, cfg.BU):
        sec.dropout = 0.2
    C, D = meta["C"], meta["D"]
    feats, label, text = tiny_inputs(meta)

    def step(seed):
        torch.manual_seed(123)
        net = FACT_CLIP(cfg, D, C, text_embeddings=torch.from_numpy(text).float())
        with torch.no_grad():
            for n, p in net.named_parameters():
                p.copy_(torch.from_numpy(pg.param_value(n, p.shape, meta["seed"])))
        net.mcriterion = MatchCriterion(cfg, C, [])
        net = net.to(DEV).train()
        torch.manual_seed(seed)
        loss, _ = net([torch.from_numpy(feats).float().to(DEV)], [torch.from_numpy(label).to(DEV)],
                      compute_loss=True)
        loss.backward()
        g = torch.cat([p.grad.reshape(-1) for p in net.parameters() if p.grad is not None])
        return loss.item(), g
    l1, g1 = step(7)
    l2, g2 = step(7)
    l3, _ = step(8)
    assert math.isfinite(l1) and torch.isfinite(g1).all()
    assert l1 == l2 and torch.equal(g1, g2)
    assert l1 != l3


def _prof_count(lib, kind):
    import ctypes
    ms, fl, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    assert lib.fx_prof_collect(kind, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by), ctypes.byref(n)) == 0
    return n.value


@pytest.mark.parametrize("fused,flat", [(1, True), (2, True), (0, True), (1, False)])
def test_mstcn_dropout_ragged_shipped_rows(fused, flat, fixed_seeds, monkeypatch):
    """The shipped yaml's frame branch shape in training (havid_view0_lh_pt_holdout.yaml: F = 256, 10
    layers, dropout 0.2, basic.py:154-171) on its ragged 4096 + 2900 batch (219 row tiles: the fused
    layer under the default 80 % fill rule).  fused: 1 = the library's fill rule, 2 = forced, 0 = the
    two-GEMM layers; flat: gradients as views of one flat buffer (the deferred batched weight gradients
    over K = rows rounded up to the 64-deep stage, the masked 1x1 gradient dB kept by the fused dX
    chain) or separate buffers (the per-layer single-stream path).  Output, input gradient and every
    weight gradient vs the float64 restatement with the SAME masks (index row * F + col of the stacked
    rows, sub-seed per layer) and the GPU's own ReLU decisions; fx_prof kind 7 proves which kernel ran."""
    from factmx import native as nx
    from factmx.dp import FlatGradReducer
    from factmx.models.basic import MSTCN
    monkeypatch.setattr(fxf, "MSTCN_FUSED_LAYERS", fused)
    lib = nx.load()
    p, nl, F = 0.2, 10, 256
    off = [0, 4096, 6996]
    rows = off[-1]
    torch.manual_seed(0)
    mod = MSTCN(64, F, 40, nl, dropout=p, ln=False, in_map=True).to(DEV).train()
    if flat:
        FlatGradReducer(mod.parameters())
    x = _r(rows, 64, seed=31)
    g = _r(rows, 40, seed=32)
    xd = x.float().to(DEV).requires_grad_(True)
    assert lib.fx_prof_enable(7, 64) == 0
    try:
        y = fxf.mstcn(mod, xd, T=0, nvid=2, seq_off=off)
        n_fwd = _prof_count(lib, 7)
        saved = y.grad_fn.saved_tensors[1].detach().double().cpu()
        assert lib.fx_prof_enable(7, 64) == 0
        (y * g.float().to(DEV)).sum().backward()
        torch.cuda.synchronize()
        n_bwd = _prof_count(lib, 7)
    finally:
        lib.fx_prof_disable()
    assert n_fwd == (nl if fused else 0), n_fwd
    assert n_bwd == (nl - 1 if fused and flat else 0), n_bwd
    seed = fixed_seeds[-1]
    n = -(-rows // 64) * 64 * F
    gates = [(saved[(nl + 1 + i) * n:(nl + 1 + i) * n + rows * F].view(rows, F) > 0).double() for i in range(nl)]
    masks = [_mask(drop_subseed(seed, i), (rows, F), p) / (1.0 - float(np.float32(p))) for i in range(nl)]
    P = {k: t.detach().double().cpu().requires_grad_(True) for k, t in mod.named_parameters()}
    xr = x.clone().requires_grad_(True)
    h = fo.linear(xr, P["conv_1x1.weight"], P["conv_1x1.bias"])
    for i in range(nl):
        q = f"layers.{i}."
        z = torch.cat([fo.dilated_conv3(h[off[v]:off[v + 1]], P[q + "conv_dilated.weight"],
                                        P[q + "conv_dilated.bias"], 2 ** i) for v in range(2)], 0) * gates[i]
        h = h + fo.linear(z, P[q + "conv_1x1.weight"], P[q + "conv_1x1.bias"]) * masks[i]
    yr = fo.linear(h, P["conv_out.weight"], P["conv_out.bias"])
    (yr * g).sum().backward()
    _close(y, yr, rtol=2e-4, atol=2e-4, what="y")
    _close(xd.grad, xr.grad, rtol=2e-4, atol=2e-4, what="dx")
    for k, t in mod.named_parameters():
        _close(t.grad, P[k].grad, rtol=2e-4, atol=2e-4, what=f"d{k}")
