"""MS-TCN++ frame branch (MSTCN2, basic.py:222-281; the Breakfast config's 'm2', BASELINE configs[0])
as one fx_mstcn2 call (GPU) against a float64 restatement (oracle.fact_oracle.mstcn2 per video, plus
the kernels' dropout mask on every layer but the last when p > 0):
  * forward output, input gradient and every weight gradient, for 1 and 2 stacked videos (the
    dilated convs zero-pad at each video's ends);
  * both weight-gradient schedules: per-layer launches (every .grad its own allocation) and the
    batched launches over all layers (gradients as views of one flat buffer, as bench.py / DP run it:
    conv_dilated_2's dilation grows with the batch index, conv_dilated_1's batch runs the layers in
    reverse through negative strides);
  * eval mode with p > 0 is bitwise the p = 0 training path."""
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


def _gpu_gates(y, nl, rows, F):
    """The GPU's ReLU decisions (r_i > 0) of every layer, read from MSTCN2Fn's saved activations
    (layout f_0..f_L, cat_0..cat_L-1 (2F), r_0..r_L-1)."""
    todo, seen = [y.grad_fn], set()
    while todo:
        node = todo.pop()
        if node is None or id(node) in seen:
            continue
        seen.add(id(node))
        if "MSTCN2Fn" in type(node).__name__:
            saved = node.saved_tensors[1]
            base = (nl + 1 + 2 * nl) * rows * F
            return [(saved[base + i * rows * F: base + (i + 1) * rows * F].view(rows, F) > 0).double().cpu()
                    for i in range(nl)]
        todo += [f for f, _ in node.next_functions]
    raise AssertionError("MSTCN2Fn node not found")


def _ref(P, x, T, nvid, nl, seed, p, gates=None):
    """fo.mstcn2 per video; layer i < nl-1 drops r_i with mask seed drop_subseed(seed, i), element
    index (global row) * F + channel (the fusion GEMM's epilogue index).  gates: take the ReLU's
    decisions from the GPU (pre-activations within fp32 rounding of 0 may land on either side)."""
    outs = []
    F = P["conv_out.weight"].shape[1]
    rows = x.shape[0]
    masks = []
    for i in range(nl - 1):
        if p > 0:
            idx = np.arange(rows, dtype=np.int64)[:, None] * F + np.arange(F, dtype=np.int64)[None, :]
            m = torch.from_numpy(drop_mask(drop_subseed(seed, i), idx, p).astype(np.float64))
            masks.append(m / (1.0 - float(np.float32(p))))
    for v in range(nvid):
        sl = slice(v * T, (v + 1) * T)
        f = fo.linear(x[sl], P["conv_1x1_in.weight"], P["conv_1x1_in.bias"])
        for i in range(nl):
            a = fo.dilated_conv3(f, P[f"conv_dilated_1.{i}.weight"], P[f"conv_dilated_1.{i}.bias"], 2 ** (nl - 1 - i))
            b = fo.dilated_conv3(f, P[f"conv_dilated_2.{i}.weight"], P[f"conv_dilated_2.{i}.bias"], 2 ** i)
            u = fo.linear(torch.cat([a, b], -1), P[f"conv_fusion.{i}.weight"], P[f"conv_fusion.{i}.bias"])
            r = torch.relu(u) if gates is None else u * gates[i][sl]
            if p > 0 and i != nl - 1:
                r = r * masks[i][sl]
            f = r + f
        outs.append(fo.linear(f, P["conv_out.weight"], P["conv_out.bias"]))
    return torch.cat(outs, 0)


def _close(a, b, tol, what):
    """max |a - b| <= tol (1 + max |b|)."""
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item()
    assert err <= tol * (1.0 + ref), f"{what}: max err {err:.3e} (ref max {ref:.3e})"


@pytest.mark.parametrize("T,nvid,F,nl,p,flat", [(300, 1, 64, 4, 0.0, False), (300, 1, 64, 4, 0.0, True),
                                                 (257, 2, 64, 5, 0.0, True), (200, 2, 64, 4, 0.3, True),
                                                 (512, 2, 512, 10, 0.0, True), (200, 1, 64, 4, 0.3, False)])
def test_mstcn2_matches_fp64(T, nvid, F, nl, p, flat, monkeypatch):
    from factmx.dp import FlatGradReducer
    from factmx.models.basic import MSTCN2
    seeds = []

    def nxt():
        seeds.append(123456789 + 7919 * len(seeds))
        return seeds[-1]
    monkeypatch.setattr(fxf, "dropout_seed", nxt)
    torch.manual_seed(0)
    cin, cout = 96, 40
    mod = MSTCN2(cin, F, cout, nl, dropout=p, in_map=True).to(DEV).train()
    red = FlatGradReducer(mod.parameters()) if flat else None
    x = _r(nvid * T, cin, seed=1)
    g = _r(nvid * T, cout, seed=2)
    xd = x.float().to(DEV).requires_grad_(True)
    y = mod(xd, T)[:, 0]
    # F = 512 x 10 layers x 1024 rows: some of the 5M fusion pre-activations lie within fp32 rounding
    # of the ReLU kink; a gate that flips between fp32 and fp64 is a true discontinuity (O(1) on
    # single gradient entries), so the fp64 restatement takes the GPU's gate decisions there
    gates = _gpu_gates(y, nl, nvid * T, F) if F > 64 else None
    (y * g.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    P = {n: t.detach().double().cpu().requires_grad_(True) for n, t in mod.named_parameters()}
    xr = x.clone().requires_grad_(True)
    yr = _ref(P, xr, T, nvid, nl, seeds[-1] if p > 0 else 0, p, gates)
    (yr * g).sum().backward()
    tol = 2e-4 if F <= 64 else 1e-3
    _close(y, yr, tol, "y")
    _close(xd.grad, xr.grad, tol, "dx")
    for n, t in mod.named_parameters():
        _close(t.grad, P[n].grad, tol, f"d{n}")
    if red is not None:
        lo = red.flat.data_ptr()
        assert all(lo <= t.grad.data_ptr() < lo + red.flat.numel() * 4 for t in mod.parameters())
    if p > 0:
        mod.eval()
        with torch.no_grad():
            ye = mod(xd, T)
            mod.dropout.p = 0.0
            mod.train()
            y0 = mod(xd, T)
        assert torch.equal(ye, y0)
