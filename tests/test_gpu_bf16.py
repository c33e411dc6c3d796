"""FX_PREC_BF16 performance mode (fx_set_gemm_precision, BASELINE configs[1]).

The bf16 kernel rounds both operands to bf16 and accumulates in fp32, so it is checked against a
float64 product of the bf16-ROUNDED inputs (fp32-accumulation tolerance), on the shapes the mode
takes (frame-level 128x64-tile launches with row-major operands, incl. the implicit dilated conv,
epilogues and split-K), plus a check that the mode really changes the arithmetic (the result sits
nearer the bf16-rounded product than the exact one) and that it is off again after the context.
The model-level deviation of FACT_CLIP in this mode is measured (and bounded loosely), not claimed
to be at parity: bench.py reports it."""
import math

import pytest
import torch

from factmx import functional as fxf
from factmx import native as nx

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64) * scale


def _bf(t):
    return t.float().to(torch.bfloat16).double()


def _rows(t, ld=None):
    o = nx.Operand()
    o.ptr = nx.ptr(t)
    o.ld = ld or t.shape[-1]
    o.conv_dir = 1
    return o


@pytest.mark.parametrize("M,N,K,split,epi,bt", [(8192, 256, 256, 1, "plain", False),
                                                (8192, 256, 768, 1, "bias_relu_resid", False),
                                                (8000, 256, 512, 1, "plain", False), (4096, 512, 1024, 2, "plain", False),
                                                (8192, 512, 2048, 1, "bias_relu_resid", False),
                                                (8192, 256, 256, 1, "plain", True), (8000, 512, 3072, 1, "plain", True)])
def test_bf16_gemm_matches_rounded_product(M, N, K, split, epi, bt):
    A = _r(M, K, seed=1)
    B = _r(N, K, seed=2, scale=K ** -0.5)          # weight (N, K): B operand rows (bt: stored (K, N))
    Ad = A.float().to(DEV)
    Bd = (B.t() if bt else B).contiguous().float().to(DEV)
    c = torch.zeros(M, N, device=DEV)
    ref_bf = _bf(A) @ _bf(B).t()
    ref = A @ B.t()
    kw = {}
    if epi == "bias_relu_resid":
        bias, resid = _r(N, seed=4), _r(M, N, seed=5)
        kw = dict(bias=bias.float().to(DEV), resid=resid.float().to(DEV), relu=1)
        ref_bf = torch.relu(ref_bf + bias + resid)
        ref = torch.relu(ref + bias + resid)
    with fxf.gemm_precision("bf16"):
        b = _rows(Bd)
        b.trans = int(bt)
        fxf.gemm(M, N, K, _rows(Ad), b, c, N, split=split, **kw)
    torch.cuda.synchronize()
    got = c.double().cpu()
    err = (got - ref_bf).abs().max().item()
    assert err <= 2e-5 * (1 + ref_bf.abs().max().item()) + 1e-6 * math.sqrt(K), err
    # the bf16 arithmetic really ran: nearer the rounded product than the exact one
    assert (got - ref).abs().max().item() > 10 * err
    assert nx.load().fx_get_gemm_precision() == nx.PREC_F32


def test_bf16_conv_gemm_matches_rounded_product():
    """Implicit dilated conv (3 taps, dilation 4, zero outside each 4096-frame video) in bf16."""
    T, nv, cin, N, dil = 4096, 2, 256, 256, 4
    M, K = T * nv, 3 * cin
    X = _r(M, cin, seed=11)
    W = _r(N, K, seed=12, scale=K ** -0.5)          # [n][tap * cin + c]
    Xd, Wd = X.float().to(DEV), W.float().to(DEV)
    a = _rows(Xd, cin)
    a.conv_taps, a.conv_cin, a.conv_dil, a.seq_len = 3, cin, dil, T
    c = torch.zeros(M, N, device=DEV)
    with fxf.gemm_precision("bf16"):
        fxf.gemm(M, N, K, a, _rows(Wd), c, N)
    torch.cuda.synchronize()
    Xb = _bf(X).view(nv, T, cin)
    cols = []
    for tap in range(3):
        s = (tap - 1) * dil
        sh = torch.zeros_like(Xb)
        if s >= 0:
            sh[:, :T - s] = Xb[:, s:]
        else:
            sh[:, -s:] = Xb[:, :T + s]
        cols.append(sh)
    ref = torch.cat(cols, 2).reshape(M, K) @ _bf(W).t()
    err = (c.double().cpu() - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err


def test_bf16_mode_fact_clip_step_deviation():
    """One FACT_CLIP forward + loss + backward at T=1024 in each mode: the bf16 frame logits stay
    within a loose bound of the fp32 ones (the mode's deviation is reported by bench.py), and the
    loss and every gradient are finite."""
    import bench
    cfg = bench.make_cfg()
    T = 1024
    net, _ = bench.build_model(cfg, bench.D_IN, bench.NCLS, DEV, seed=0)
    net.train()
    f, lab = bench.make_video(T, bench.D_IN, bench.NCLS, cfg, seed=1)
    seqs = [torch.from_numpy(f).to(DEV)]
    labels = [torch.from_numpy(lab).to(DEV)]

    def run():
        net.zero_grad(set_to_none=True)
        loss, _ = net(seqs, labels, compute_loss=True)
        loss.backward()
        logits = net.block_list[-1].frame_clogit.detach().clone()
        grads = [p.grad.detach().clone() for p in net.parameters() if p.grad is not None]
        return float(loss), logits, grads

    l32, z32, g32 = run()
    with fxf.gemm_precision("bf16"):
        l16, z16, g16 = run()
    assert math.isfinite(l16) and all(torch.isfinite(g).all() for g in g16)
    dev = (z16 - z32).abs().max().item()
    assert dev < 0.25 * (1 + z32.abs().max().item()), dev
    assert abs(l16 - l32) < 0.05 * (1 + abs(l32))
