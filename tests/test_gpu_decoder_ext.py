"""The fused action-token decoder (fx_decoder_*) beyond round 2's envelope (GPU):

* more than 64 tokens per video (the reference yamls use ntoken 75 / 200 / 300:
  havid_view0_lh_pt_holdout.yaml:75, egoprocel.yaml, epic-kitchens.yaml) -- the self-attention then
  runs on the attention-over-T kernels in query blocks of 64, the cross-attention in query blocks;
* training dropout inside the fused decoder (SALayer / SCALayer dropout1/2/3, FFN hidden, attention
  probabilities, basic.py:444-449, 498-522) with the documented counter-based masks
  (include/factmx.h fx_decoder_params.seed), against a float64 restatement applying the same masks;
* ragged videos: frame memories of different lengths (fx_decoder_params.mem_off).

Every case checks the output and every input / parameter gradient of a 2-video lockstep call against
the fp64 reference, run per video as the reference does.
"""
import math
import zlib

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


def _keep(seed, idx, p):
    """keep / (1 - p) of the kernels' mask at index array idx (float64)."""
    if p <= 0:
        return torch.ones(idx.shape, dtype=torch.float64)
    return torch.from_numpy(drop_mask(seed, idx, p).astype(np.float64)) / (1.0 - float(np.float32(p)))


class _Masks:
    """The fused decoder's dropout masks (fx_decoder_params.seed): site s of layer l has seed
    fx_drop_subseed(seed, 8 l + s); branch masks index r * width + c over ALL token rows; attention
    probabilities (query_row * nhead + head) * key_rows_total + key_row."""

    def __init__(self, seed, pd, pa, R, nh):
        self.seed, self.pd, self.pa, self.R, self.nh = seed, pd, pa, R, nh

    def branch(self, l, site, width):
        idx = np.arange(self.R)[:, None] * width + np.arange(width)[None, :]
        return _keep(drop_subseed(self.seed, 8 * l + site), idx, self.pd)

    def probs(self, l, site, qrows, krows, ktot):
        """(nh, len(qrows), len(krows)) keep-scales for global query / key row index arrays."""
        q = np.asarray(qrows)[None, :, None]
        h = np.arange(self.nh)[:, None, None]
        k = np.asarray(krows)[None, None, :]
        return _keep(drop_subseed(self.seed, 8 * l + site), (q * self.nh + h) * ktot + k, self.pa)


def _mha_masked(P, p, q_in, k_in, v_in, nh, keep):
    """fo.mha with keep-scales (nh, Lq, Lk) multiplying the attention probabilities."""
    E = q_in.shape[-1]
    hd = E // nh
    bi = P[p + "in_proj_bias"]
    if (p + "in_proj_weight") in P:
        W = P[p + "in_proj_weight"]
        wq, wk, wv = W[:E], W[E:2 * E], W[2 * E:]
    else:
        wq, wk, wv = P[p + "q_proj_weight"], P[p + "k_proj_weight"], P[p + "v_proj_weight"]
    q, k, v = fo.linear(q_in, wq, bi[:E]), fo.linear(k_in, wk, bi[E:2 * E]), fo.linear(v_in, wv, bi[2 * E:])
    L, S = q.shape[0], k.shape[0]
    qh = q.reshape(L, nh, hd).transpose(0, 1)
    kh = k.reshape(S, nh, hd).transpose(0, 1)
    vh = v.reshape(S, nh, hd).transpose(0, 1)
    att = fo.softmax(qh @ kh.transpose(1, 2) / math.sqrt(hd)) * keep
    o = (att @ vh).transpose(0, 1).reshape(L, E)
    return fo.linear(o, P[p + "out_proj.weight"], P[p + "out_proj.bias"])


def _ref_decoder(P, cross, tgt, qpos, mem, mpos, Q, moff, nl, nh, M):
    """SCADecoder / SADecoder forward (basic.py:494-523 / 429-452, 542-557 / 578-593) over stacked
    videos of Q tokens (memory rows moff[v]:moff[v+1]), dropout from _Masks M."""
    nvid = tgt.shape[0] // Q
    A = tgt.shape[1]
    x = tgt
    for l in range(nl):
        p = f"layers.{l}."
        outs = []
        for v in range(nvid):
            r = slice(v * Q, (v + 1) * Q)
            q = fo.add_pos(x[r], qpos[r])
            rows = np.arange(v * Q, (v + 1) * Q)
            keep = M.probs(l, 0, rows, rows, nvid * Q)
            sa = _mha_masked(P, p + ("self_attn." if cross else "multihead_attn."), q, q, x[r], nh, keep)
            outs.append(sa)
        sa = torch.cat(outs)
        t = fo.layer_norm(x + sa * M.branch(l, 1, A), P[p + "norm1.weight"], P[p + "norm1.bias"])
        if cross:
            outs = []
            for v in range(nvid):
                r = slice(v * Q, (v + 1) * Q)
                m = slice(moff[v], moff[v + 1])
                keep = M.probs(l, 2, np.arange(v * Q, (v + 1) * Q), np.arange(moff[v], moff[v + 1]), moff[-1])
                outs.append(_mha_masked(P, p + "multihead_attn.", fo.add_pos(t[r], qpos[r]),
                                        fo.add_pos(mem[m], None if mpos is None else mpos[m]), mem[m], nh, keep))
            t = fo.layer_norm(t + torch.cat(outs) * M.branch(l, 3, A), P[p + "norm2.weight"], P[p + "norm2.bias"])
        FF = P[p + "linear1.weight"].shape[0]
        h = torch.relu(fo.linear(t, P[p + "linear1.weight"], P[p + "linear1.bias"])) * M.branch(l, 4, FF)
        ff = fo.linear(h, P[p + "linear2.weight"], P[p + "linear2.bias"]) * M.branch(l, 5, A)
        n3 = "norm3." if cross else "norm2."
        x = fo.layer_norm(t + ff, P[p + n3 + "weight"], P[p + n3 + "bias"])
    if cross:
        x = fo.layer_norm(x, P["norm.weight"], P["norm.bias"])
    return fo.linear(x, P["out_linear.weight"], P["out_linear.bias"])


def _close(a, b, rtol, atol, what):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item()
    assert err <= atol + rtol * ref, f"{what}: max err {err:.3e} (ref max {ref:.3e})"


def _build(cross, A, nh, FF, nl, Hm, out_dim, p):
    from factmx.models.basic import SADecoder, SALayer, SCADecoder, SCALayer
    torch.manual_seed(0)
    if cross:
        lyr = SCALayer(A, Hm, nh, FF, dropout=p, attn_dropout=p)
        dec = SCADecoder(A, A, out_dim, lyr, nl, norm=torch.nn.LayerNorm(A))
    else:
        lyr = SALayer(A, nh, dim_feedforward=FF, dropout=p, attn_dropout=p)
        dec = SADecoder(A, A, out_dim, lyr, nl)
    with torch.no_grad():      # layers differ (the reference clones one layer; distinct values test indexing)
        for n, t in dec.named_parameters():
            is_ln_w = n.endswith("weight") and n.split(".")[-2].startswith("norm")
            t.copy_(_r(*t.shape, seed=zlib.crc32(n.encode()) % 10007, scale=0.6 / math.sqrt(t.shape[-1])) +
                    (1.0 if is_ln_w else 0.0))
    return dec.to(DEV)


CASES = [
    # cross, tokens per video, memory rows per video, dropout
    (True, 75, (300, 300), 0.0),
    (True, 75, (300, 220), 0.2),
    (True, 32, (257, 400), 0.2),
    (False, 75, None, 0.2),
    (False, 130, None, 0.0),
    (False, 32, None, 0.2),
]


def _tok_launches(lib):
    import ctypes
    ms, fl, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
    assert lib.fx_prof_collect(8, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by), ctypes.byref(n)) == 0
    return n.value


@pytest.mark.parametrize("cross,Q,T,p", CASES)
def test_fused_decoder_tokens_dropout_ragged(cross, Q, T, p, monkeypatch):
    _decoder_case(cross, Q, T, p, monkeypatch, 64, 4, 96, expect_tok=False)


# shapes of the persistent token kernel (tokdec.hip): head dim 32, <= 32 tokens per video
TOK_CASES = [
    (True, 32, (300, 220), 0.2),
    # a one-chunk frame memory beside a 5000-frame one: more key chunks than the attention's in-launch
    # merge takes, so the merge launch runs over both videos
    (True, 32, (33, 5000), 0.0),
    (True, 20, (257, 257), 0.0),
    (True, 7, (64, 90), 0.2),
    (False, 32, None, 0.2),
    (False, 17, None, 0.0),
]


@pytest.mark.parametrize("cross,Q,T,p", TOK_CASES)
def test_token_kernel_decoder_dropout_ragged(cross, Q, T, p, monkeypatch):
    """The persistent token kernel's programs (forward and backward, LayerNorm staged into the products,
    in-projection + self-attention items, dropout at every site, ragged frame memory) vs the float64
    masked restatement, and fx_prof kind 8 proves the kernel ran."""
    _decoder_case(cross, Q, T, p, monkeypatch, 128, 4, 192, expect_tok=True)


def _decoder_case(cross, Q, T, p, monkeypatch, A, nh, FF, expect_tok):
    from factmx import native as nx
    seeds = []

    def nxt():
        seeds.append(0x5DEECE66D * (len(seeds) + 3) % 2 ** 62)
        return seeds[-1]
    monkeypatch.setattr(fxf, "dropout_seed", nxt)
    nl, Hm, out_dim, nvid = 2, 96, 80, 2
    dec = _build(cross, A, nh, FF, nl, Hm, out_dim, p).train()
    R = nvid * Q
    moff = [0] + [int(x) for x in np.cumsum(T)] if cross else None
    tgt, qpos, g = _r(R, A, seed=1), _r(R, A, seed=2, scale=0.5), _r(R, out_dim, seed=3)
    mem = _r(moff[-1], Hm, seed=4) if cross else None
    mpos = _r(moff[-1], Hm, seed=5, scale=0.5) if cross else None
    dt = [t.float().to(DEV).requires_grad_(True) for t in (tgt, qpos)]
    dm = [t.float().to(DEV).requires_grad_(True) for t in (mem, mpos)] if cross else [None, None]
    ragged = cross and T[0] != T[1]
    lib = nx.load()
    assert lib.fx_prof_enable(8, 64) == 0
    try:
        y = fxf.decoder(dec, dt[0], dm[0], pos=dm[1], query_pos=dt[1], nvid=nvid, mem_off=moff if ragged else None)
        (y * g.float().to(DEV)).sum().backward()
        fxf.side_join()
        torch.cuda.synchronize()
        ntok = _tok_launches(lib)
    finally:
        lib.fx_prof_disable()
    assert (ntok > 0) == expect_tok, ntok
    fxf.check_device_status()
    assert len(seeds) == (1 if p > 0 else 0)
    M = _Masks(seeds[-1] if seeds else 0, p, p, R, nh)
    P = {n: t.detach().double().cpu().requires_grad_(True) for n, t in dec.named_parameters()}
    rt = [t.clone().requires_grad_(True) for t in (tgt, qpos)]
    rm = [t.clone().requires_grad_(True) for t in (mem, mpos)] if cross else [None, None]
    yr = _ref_decoder(P, cross, rt[0], rt[1], rm[0], rm[1], Q, moff, nl, nh, M)
    (yr * g).sum().backward()
    tol = dict(rtol=2e-4, atol=2e-4)
    _close(y, yr, what="out", **tol)
    _close(dt[0].grad, rt[0].grad, what="dtgt", **tol)
    _close(dt[1].grad, rt[1].grad, what="dqpos", **tol)
    if cross:
        _close(dm[0].grad, rm[0].grad, what="dmem", **tol)
        _close(dm[1].grad, rm[1].grad, what="dmpos", **tol)
    for n, t in dec.named_parameters():
        _close(t.grad, P[n].grad, what=f"d{n}", rtol=5e-4, atol=5e-4)


def test_dropout_eval_and_p0_are_the_plain_path():
    """Eval mode with p > 0, and p = 0 in training, run bitwise the no-dropout decoder."""
    dec = _build(True, 64, 4, 96, 2, 96, 80, 0.2)
    tgt = _r(150, 64, seed=1).float().to(DEV)
    qpos = _r(150, 64, seed=2).float().to(DEV)
    mem = _r(600, 96, seed=4).float().to(DEV)
    with torch.no_grad():
        dec.eval()
        ye = fxf.decoder(dec, tgt, mem, pos=None, query_pos=qpos, nvid=2)
        for m in dec.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
            if isinstance(m, torch.nn.MultiheadAttention):
                m.dropout = 0.0
        dec.train()
        y0 = fxf.decoder(dec, tgt, mem, pos=None, query_pos=qpos, nvid=2)
    assert torch.equal(ye, y0)
