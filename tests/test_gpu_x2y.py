"""X2Y_map (basic.py:349-389) through X2YFn on the GPU against the fp64 oracle (fo.x2y), per video of a
stacked ragged batch: the a2f direction (keys = action tokens: the fused one-launch core of
x2y_core.hip for <= 64 keys, including two key blocks at 40 keys, and the grouped-GEMM path past 64
keys), the f2a direction (keys = frames), and the core switched off (FX_X2Y_FUSED=0 equivalent: the
grouped path) -- out, logit and attn forward, every input / weight gradient backward."""
import math

import pytest
import torch

from factmx import functional as fxf
from oracle import fact_oracle as fo

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, A, D2 = 512, 256, 256   # head dim (X_K / X_V / Y_Q out), x feature dim, y feature dim


def _params(xdim, ydim, outdim, seed):
    g = torch.Generator().manual_seed(seed)
    P = {}
    for n, shp in (("X_K.weight", (H, xdim)), ("X_K.bias", (H,)), ("X_V.weight", (H, xdim)), ("X_V.bias", (H,)),
                   ("Y_Q.weight", (H, ydim)), ("Y_Q.bias", (H,)), ("Y_W.weight", (outdim, ydim + H)),
                   ("Y_W.bias", (outdim,))):
        fan = shp[1] if len(shp) > 1 else 1
        P[n] = (torch.randn(*shp, generator=g, dtype=torch.float64) / math.sqrt(fan)).float().double()
    return P


@pytest.mark.parametrize("direction,nq,Ts", [("a2f", 32, (700, 413)), ("a2f", 40, (300, 257)),
                                             ("a2f", 64, (129, 64)), ("a2f", 75, (300, 200)),
                                             ("f2a", 32, (700, 413)), ("f2a", 40, (300, 257, 65)),
                                             ("f2a", 64, (64, 1)), ("f2a", 75, (200, 90)),
                                             ("a2f", 32, (1,)), ("f2a", 7, (3000,))])
def test_x2y_vs_oracle(direction, nq, Ts):
    g = torch.Generator().manual_seed(7)
    nv = len(Ts)
    tok = [torch.randn(nq, A, generator=g, dtype=torch.float64).float().double() for _ in Ts]
    frm = [torch.randn(T, D2, generator=g, dtype=torch.float64).float().double() for T in Ts]
    tpos = [0.5 * torch.randn(nq, A, generator=g, dtype=torch.float64).float().double() for _ in Ts]
    fpos = [0.5 * torch.randn(T, D2, generator=g, dtype=torch.float64).float().double() for T in Ts]
    if direction == "a2f":           # X = tokens, Y = frames
        Xs, Ys, Xps, Yps, xdim, ydim = tok, frm, tpos, fpos, A, D2
    else:
        Xs, Ys, Xps, Yps, xdim, ydim = frm, tok, fpos, tpos, D2, A
    outdim = 192
    P = _params(xdim, ydim, outdim, seed=3)
    xl, yl = [0], [0]
    for X, Y in zip(Xs, Ys):
        xl.append(xl[-1] + X.shape[0])
        yl.append(yl[-1] + Y.shape[0])
    cat = lambda ts: torch.cat(ts).float().to(DEV).requires_grad_(True)   # noqa: E731
    X, Y, Xp, Yp = cat(Xs), cat(Ys), cat(Xps), cat(Yps)
    W = {n: t.float().to(DEV).requires_grad_(True) for n, t in P.items()}
    rows = (xl, yl) if nv > 1 else None
    out, logit, attn = fxf.X2YFn.apply(X, Y, Xp, Yp, rows, W["X_K.weight"], W["X_K.bias"], W["X_V.weight"],
                                       W["X_V.bias"], W["Y_Q.weight"], W["Y_Q.bias"], W["Y_W.weight"],
                                       W["Y_W.bias"], 0.0, 0)
    gen = torch.Generator().manual_seed(9)
    gout = torch.randn(out.shape, generator=gen, dtype=torch.float64)
    glog = torch.randn(logit.shape, generator=gen, dtype=torch.float64)
    loss = (out.double() * gout.to(DEV)).sum() + (logit.double() * glog.to(DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    # oracle per video (fp64), same upstream gradients
    Pr = {n: t.clone().requires_grad_(True) for n, t in P.items()}
    Xr = [t.clone().requires_grad_(True) for t in Xs]
    Yr = [t.clone().requires_grad_(True) for t in Ys]
    Xpr = [t.clone().requires_grad_(True) for t in Xps]
    Ypr = [t.clone().requires_grad_(True) for t in Yps]
    lo, ao, total, a0 = [], [], 0, 0
    for v in range(nv):
        o, lg, at = fo.x2y(Pr, "", Xr[v], Yr[v], Xpr[v], Ypr[v])
        n = lg.numel()
        total = total + (o * gout[yl[v]:yl[v + 1]]).sum() + (lg.reshape(-1) * glog.reshape(-1)[a0:a0 + n]).sum()
        lo.append(lg.reshape(-1))
        ao.append(at.reshape(-1))
        a0 += n
    total.backward()
    ref_out = None
    with torch.no_grad():
        ref_out = torch.cat([fo.x2y(P, "", Xs[v], Ys[v], Xps[v], Yps[v])[0] for v in range(nv)])

    def close(got, ref, tol, what):
        got = got.detach().double().cpu().reshape(ref.shape)
        err = (got - ref).abs().max().item()
        assert err <= tol * (1 + ref.abs().max().item()), (what, err)

    close(out, ref_out, 1e-4, "out")
    close(logit, torch.cat(lo).detach(), 1e-4, "logit")
    close(attn, torch.cat(ao).detach(), 1e-5, "attn")
    close(X.grad, torch.cat([t.grad for t in Xr]), 1e-4, "dX")
    close(Y.grad, torch.cat([t.grad for t in Yr]), 1e-4, "dY")
    close(Xp.grad, torch.cat([t.grad for t in Xpr]), 1e-4, "dXpos")
    close(Yp.grad, torch.cat([t.grad for t in Ypr]), 1e-4, "dYpos")
    for n in P:
        close(W[n].grad, Pr[n].grad, 2e-4, n)
