"""Host-side helpers of the lockstep path (CPU): per-video chunk views and loss-term summation
give the same values and gradients as the slicing / `+` chains they replace."""
import pytest
import torch

from factmx.models.blocks import _sum_terms, _VideoBatch


@pytest.mark.parametrize("Ts", [[5, 5, 5], [5, 3, 7]])
def test_video_chunks_match_slices_in_value_and_grad(Ts):
    """Per-video frame / token chunks of a lockstep batch (equal or ragged video lengths)."""
    vb = _VideoBatch(nvid=3, Ts=Ts, Q=2)
    assert vb.ragged == (len(set(Ts)) > 1) and vb.f_off == [0, Ts[0], Ts[0] + Ts[1], sum(Ts)]
    n = sum(Ts)
    x = torch.randn(n, 4, dtype=torch.float64, requires_grad=True)
    y = torch.randn(6, 3, dtype=torch.float64, requires_grad=True)
    w = torch.randn(n, 4, dtype=torch.float64)
    # only videos 0 and 2 contribute to the loss (video 1's chunk gets no gradient)
    xs, ys = vb.frames(x), vb.tokens(y)
    loss = (xs[0] * w[vb.fr(0)]).sum() + (xs[2] ** 2).sum() + ys[1][:, :-1].sum()
    loss.backward()
    gx, gy = x.grad.clone(), y.grad.clone()
    x.grad = y.grad = None
    ref = (x[vb.fr(0)] * w[vb.fr(0)]).sum() + (x[vb.fr(2)] ** 2).sum() + y[vb.tk(1), :-1].sum()
    ref.backward()
    assert torch.equal(gx, x.grad) and torch.equal(gy, y.grad)
    assert torch.equal(gx[vb.fr(1)], torch.zeros(Ts[1], 4, dtype=torch.float64))


def test_sum_terms():
    a = torch.tensor(1.5, requires_grad=True)
    b = torch.tensor([2.25], requires_grad=True)
    s = _sum_terms([a, b, 0.25])
    assert float(s) == 4.0
    s.backward()
    assert float(a.grad) == 1.0 and float(b.grad[0]) == 1.0
    assert _sum_terms([0.5, 0.25]) == 0.75
    assert _sum_terms([a]) is a
