"""The transcript-conditioned GRU action branch (reference basic.py:283-308, ``ActionUpdate_GRU``) on the
library's BiGRU (GPU): a 2-layer bidirectional GRU + LayerNorm + output map over the action tokens,
against the same module evaluated by plain PyTorch fp32 on the CPU (``nn.GRU``, ``nn.LayerNorm``,
``nn.Linear``) -- output and every parameter / input gradient within 1e-4 (scaled by the tensor's
magnitude).  In training mode the inter-layer dropout is nn.GRU's: off at p = 0, and a p > 0 run keeps
the values finite and the kept positions' pattern (the second layer sees zeros)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_ref(mod, tgt):
    out, _ = mod.gru(tgt)
    out = mod.layernorm(out)
    return mod.out_map(out)


def _close(a, b, tol=1e-4):
    scale = max(b.abs().max().item(), 1.0)
    return (a - b).abs().max().item() <= tol * scale


@pytest.mark.parametrize("n_layers,out_map", [(1, False), (2, True)])
def test_action_update_gru_matches_torch(n_layers, out_map):
    from factmx.models import basic
    torch.manual_seed(3)
    a_dim, hid, L = 256, 384, 30
    mod = basic.ActionUpdate_GRU(a_dim, a_dim, hid if out_map else a_dim, n_layers, dropout=0.0, out_map=out_map)
    ref = basic.ActionUpdate_GRU(a_dim, a_dim, hid if out_map else a_dim, n_layers, dropout=0.0, out_map=out_map)
    ref.load_state_dict(mod.state_dict())
    mod = mod.cuda().train()
    ref = ref.train()
    x = torch.randn(L, 1, a_dim)
    g = torch.randn(L, 1, hid if out_map else a_dim)
    xg = x.cuda().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    y = mod(xg, None)
    yr = _torch_ref(ref, xr)
    assert y.shape == yr.shape
    assert _close(y.detach().cpu(), yr.detach())
    (y * g.cuda()).sum().backward()
    (yr * g).sum().backward()
    assert _close(xg.grad.cpu(), xr.grad)
    for (n, p), (_, pr) in zip(mod.named_parameters(), ref.named_parameters()):
        assert _close(p.grad.cpu(), pr.grad), n


def test_action_update_gru_interlayer_dropout():
    from factmx import functional as fxf
    torch.manual_seed(5)
    gru = torch.nn.GRU(64, 32, 2, dropout=0.5, bidirectional=True).cuda().train()
    x = torch.randn(40, 64, device="cuda", requires_grad=True)
    y = fxf.gru(gru, x)
    y.sum().backward()
    assert y.shape == (40, 64) and torch.isfinite(y).all() and torch.isfinite(x.grad).all()
    gru.eval()                 # eval: no dropout, deterministic and equal to torch's own GRU
    with torch.no_grad():
        ye = fxf.gru(gru, x)
        yt, _ = gru(x.unsqueeze(1))
    assert _close(ye, yt.squeeze(1))
