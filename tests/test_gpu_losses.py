"""Fused loss kernels (fx_class_loss_*, fx_attn_loss_*) vs the reference formulas of
fact_clip/models/loss.py written with float64 torch ops (GPU)."""
import pytest
import torch
import torch.nn.functional as F

from factmx import functional as fxf

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _smooth(logit):          # loss.py:8-18 on a (1, T, C) tensor
    lp = F.log_softmax(logit, dim=2)
    d = lp[:, 1:] - lp[:, :-1]
    return torch.clamp(d * d, min=0, max=16).mean()


def _close(a, b, tol, what):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = (a - b).abs().max().item()
    assert err <= tol * max(1.0, b.abs().max().item()), f"{what}: {err:.3e}"


@pytest.mark.parametrize("R,C,soft,sm,scale", [(4096, 75, False, 5.0, 1.0), (300, 75, True, 0.0, 1.0),
                                               (37, 11, False, 5.0, 3.0), (2, 5, False, 1.0, 30.0)])
def test_class_loss(R, C, soft, sm, scale):
    g = torch.Generator().manual_seed(R + C)
    x = torch.randn(R, C, generator=g, dtype=torch.float64) * scale
    y = torch.randint(0, C, (R,), generator=g)
    w = torch.rand(C, generator=g, dtype=torch.float64) + 0.5
    z = torch.rand(R, C, generator=g, dtype=torch.float64) if soft else None
    if soft:
        z = z / z.sum(1, keepdim=True)
    xr = x.clone().requires_grad_(True)
    lp = F.log_softmax(xr, -1)
    tgt = z if soft else F.one_hot(y, C).double()
    ce = (-lp * tgt * w).sum() / tgt.sum()
    ref = 0.7 * ce + sm * _smooth(xr.unsqueeze(0)) if sm else 0.7 * ce
    ref.backward()
    xd = x.float().to(DEV).requires_grad_(True)
    c_sm = sm / ((R - 1) * C) if sm else 0.0
    out = fxf.ClassLossFn.apply(xd, None if soft else y.to(DEV), None if not soft else z.float().to(DEV),
                                w.float().to(DEV), 0.7 / float(tgt.sum()), c_sm)
    (out * 1.3).backward()
    _close(out, ref, 2e-5, "loss")
    _close(xd.grad, xr.grad * 1.3, 2e-4, "dx")


@pytest.mark.parametrize("R,Q,K,axis,sm,transposed", [(4096, 32, 10, 1, 5.0, False), (4096, 32, 10, 0, 5.0, True),
                                                      (26, 32, 9, 0, 0.0, True), (26, 32, 9, 1, 0.0, False),
                                                      (7, 5, 5, 1, 2.0, False)])
def test_attn_loss(R, Q, K, axis, sm, transposed):
    g = torch.Generator().manual_seed(R * Q + K)
    S = K
    base = torch.randn(Q, R, generator=g, dtype=torch.float64) * 2 if transposed else \
        torch.randn(R, Q, generator=g, dtype=torch.float64) * 2
    aind = torch.randperm(Q, generator=g)[:K].sort().values
    sind = torch.randperm(S, generator=g)
    z = torch.rand(R, S, generator=g, dtype=torch.float64)
    sw = torch.rand(S, generator=g, dtype=torch.float64) + 0.5
    denom = float(z.sum())
    br = base.clone().requires_grad_(True)
    L = br.t() if transposed else br
    lp = torch.log_softmax(L[:, aind], dim=axis)
    ref = (-lp * z[:, sind] * sw).sum() / denom
    if sm:
        ref = ref + sm * _smooth(L.unsqueeze(0))
    ref.backward()
    bd = base.float().to(DEV).requires_grad_(True)
    Ld = bd.t() if transposed else bd
    c_sm = sm / ((R - 1) * Q) if sm else 0.0
    out = fxf.AttnLossFn.apply(Ld, z.float().to(DEV).contiguous(), aind.tolist(), sind.tolist(), sw.tolist(), axis,
                               1.0 / denom, c_sm)
    out.backward()
    _close(out, ref, 2e-5, "loss")
    _close(bd.grad, br.grad, 2e-4, "dL")
