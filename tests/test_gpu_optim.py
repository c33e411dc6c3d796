"""Fused clip_grad_norm_ + Adam on flat buffers (fx_adam_step) vs torch.nn.utils.clip_grad_norm_ +
torch.optim.Adam (scripts/train.py:265-267) on the same parameters and gradients (GPU)."""
import pytest
import torch

from factmx.optim import FusedAdam, clip_grad_norm_flat_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _params(seed, shapes):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(*s, generator=g).to(DEV)) for s in shapes]


# odd sizes exercise the scalar tail; (1,) a lone bias
SHAPES = [(7, 5), (256, 256, 3), (1,), (513,), (33, 17)]


@pytest.mark.parametrize("max_norm,wd,gscale", [(10.0, 0.0, 1.0), (10.0, 0.0, 50.0), (None, 0.01, 1.0),
                                                (0.5, 0.0, 3.0)])
def test_fused_adam_matches_torch(max_norm, wd, gscale):
    ref = _params(0, SHAPES)
    mine = _params(0, SHAPES)
    opt_ref = torch.optim.Adam(ref, lr=1e-3, weight_decay=wd)
    opt = FusedAdam(mine, lr=1e-3, weight_decay=wd, max_grad_norm=max_norm)
    g = torch.Generator().manual_seed(1)
    for step in range(4):
        grads = [torch.randn(*s, generator=g).to(DEV) * gscale for s in SHAPES]
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        for p, gr in zip(mine, grads):
            p.grad.copy_(gr)
        if max_norm:
            n_ref = torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt_ref.step()
        opt.step()
        torch.cuda.synchronize()
        if max_norm:
            assert abs(opt.total_norm.item() - n_ref.item()) <= 1e-5 * n_ref.item()
        for a, b in zip(mine, ref):
            assert torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-7), "clipped grad differs"
            err = (a.detach() - b.detach()).abs().max().item()
            assert err <= 2e-6, f"step {step}: param err {err}"


def test_clip_grad_norm_flat():
    g = torch.Generator().manual_seed(3)
    flat = (torch.randn(100003, generator=g) * 0.1).to(DEV)
    ref = flat.clone()
    n_ref = torch.linalg.vector_norm(ref)
    ref.mul_(torch.clamp(1.0 / (n_ref + 1e-6), max=1.0))
    n = clip_grad_norm_flat_(flat, 1.0)
    torch.cuda.synchronize()
    assert abs(n.item() - n_ref.item()) <= 1e-5 * n_ref.item()
    assert torch.allclose(flat, ref, rtol=1e-5, atol=1e-8)
