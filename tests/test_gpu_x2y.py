"""X2Y_map (basic.py:349-389) through X2YFn on the GPU against the fp64 oracle (fo.x2y), per video of a
stacked ragged batch: the a2f direction (keys = action tokens: the fused one-launch core of
x2y_core.hip for <= 64 keys, including two key blocks at 40 keys, and the grouped-GEMM path past 64
keys), the f2a direction (keys = frames), and the core switched off (FX_X2Y_FUSED=0 equivalent: the
grouped path) -- out, logit and attn forward, every input / weight gradient backward, with random
upstream gradients on all three outputs.  The reference's losses read attn_logit only (blocks.py:372-377,
491-492; attn feeds the matching and eval, blocks.py:96, 243-281), so X2YFn marks attn non-differentiable;
the C entry point still takes a dattn (fx_x2y_bwd), and this test reaches it through a subclass whose
attn output is differentiable, so the cores' dP += dattn paths are checked against the oracle too.  The
fused f2a backward core runs by default for calls of >= 64 key chunks (the 4096 + 300 frame case); every
f2a case runs again through it in a child process (FX_X2Y_F2A_BWD=1; library knobs are read once per
process)."""
import math
import os
import subprocess
import sys

import pytest
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_ROOT, os.path.join(_ROOT, "fact-clip_amd")):     # (the child process has no conftest)
    if _p not in sys.path:
        sys.path.insert(0, _p)
from factmx import functional as fxf  # noqa: E402
from oracle import fact_oracle as fo  # noqa: E402

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
                                             ("a2f", 32, (1,)), ("f2a", 7, (3000,)),
                                             ("f2a", 32, (4096, 300))])
def test_x2y_vs_oracle(direction, nq, Ts):
    check_x2y(direction, nq, Ts)


@pytest.mark.parametrize("one_launch", ["1", "0"])
def test_x2y_f2a_fused_backward_vs_oracle(one_launch):
    """The f2a cases again with the fused f2a backward core switched on for every call, as one launch
    with a grid barrier between the dP and dlogit passes (default) and as two launches
    (FX_X2Y_F2A_ONE=0); child processes: the knobs are read when the library loads."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FX_X2Y_F2A_BWD="1", FX_X2Y_F2A_ONE=one_launch)
    p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), "f2a"], env=env, cwd=root, timeout=240)
    assert p.returncode == 0, p.returncode


class _X2YAttnGrad(fxf.X2YFn):
    """X2YFn with a differentiable attn output (test only): backward receives dattn."""

    @staticmethod
    def forward(ctx, *args):
        outs = fxf.X2YFn.forward(ctx, *args)
        ctx.non_differentiable = ()
        return outs


def test_x2y_attn_not_differentiable_in_product():
    x = torch.randn(5, A, device=DEV, requires_grad=True)
    y = torch.randn(7, D2, device=DEV, requires_grad=True)
    P = {n: t.float().to(DEV).requires_grad_(True) for n, t in _params(A, D2, 8, seed=1).items()}
    _, logit, attn = fxf.X2YFn.apply(x, y, None, None, None, P["X_K.weight"], P["X_K.bias"], P["X_V.weight"],
                                     P["X_V.bias"], P["Y_Q.weight"], P["Y_Q.bias"], P["Y_W.weight"], P["Y_W.bias"],
                                     0.0, 0)
    assert logit.requires_grad and not attn.requires_grad


CASES = [("a2f", 32, (700, 413)), ("a2f", 40, (300, 257)), ("a2f", 64, (129, 64)), ("a2f", 75, (300, 200)),
         ("f2a", 32, (700, 413)), ("f2a", 40, (300, 257, 65)), ("f2a", 64, (64, 1)), ("f2a", 75, (200, 90)),
         ("a2f", 32, (1,)), ("f2a", 7, (3000,))]


def check_x2y(direction, nq, Ts):
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
    out, logit, attn = _X2YAttnGrad.apply(X, Y, Xp, Yp, rows, W["X_K.weight"], W["X_K.bias"], W["X_V.weight"],
                                       W["X_V.bias"], W["Y_Q.weight"], W["Y_Q.bias"], W["Y_W.weight"],
                                       W["Y_W.bias"], 0.0, 0)
    gen = torch.Generator().manual_seed(9)
    gout = torch.randn(out.shape, generator=gen, dtype=torch.float64)
    glog = torch.randn(logit.shape, generator=gen, dtype=torch.float64)
    gatt = torch.randn(attn.shape, generator=gen, dtype=torch.float64)
    loss = ((out.double() * gout.to(DEV)).sum() + (logit.double() * glog.to(DEV)).sum() +
            (attn.double() * gatt.to(DEV)).sum())
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
        total = (total + (o * gout[yl[v]:yl[v + 1]]).sum() + (lg.reshape(-1) * glog.reshape(-1)[a0:a0 + n]).sum() +
                 (at.reshape(-1) * gatt.reshape(-1)[a0:a0 + n]).sum())
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


if __name__ == "__main__":      # child of test_x2y_f2a_fused_backward_vs_oracle: python tests/test_gpu_x2y.py f2a
    for d, nq, Ts in CASES:
        if d == sys.argv[1]:
            check_x2y(d, nq, Ts)
            print("ok", d, nq, Ts, flush=True)
