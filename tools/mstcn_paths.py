"""Diagnostic: MS-TCN F=256 fwd/bwd vs the fp64 oracle for every (forward, backward) path pair
(FX_MSTCN_FUSED per phase); every error above 1e-4 printed (ReLU kink flips show up here)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402
from factmx.models.basic import MSTCN  # noqa: E402
from oracle import fact_oracle as fo  # noqa: E402


def rel(a, b):
    return ((a.double().cpu() - b).abs().max() / b.abs().max()).item()


for T, nvid, nl in ((8192, 1, 2),):
    for fused in ("11", "00", "10", "01"):
        os.environ["FX_MSTCN_FUSED"] = fused[0]
        torch.manual_seed(0)
        mod = MSTCN(96, 256, 40, nl, dropout=0.0, ln=False, in_map=True).cuda().train()
        rows = T * nvid
        g = torch.Generator().manual_seed(11)
        x = torch.randn(rows, 96, generator=g, dtype=torch.float64)
        gg = torch.randn(rows, 40, generator=g, dtype=torch.float64)
        xd = x.float().cuda().requires_grad_(True)
        y = fxf.mstcn(mod, xd, T=T, nvid=nvid)
        os.environ["FX_MSTCN_FUSED"] = fused[1]
        (y * gg.float().cuda()).sum().backward()
        torch.cuda.synchronize()
        P = {n: t.detach().double().cpu().requires_grad_(True) for n, t in mod.named_parameters()}
        xr = x.clone().requires_grad_(True)
        yr = torch.cat([fo.mstcn(P, "", xr[v * T:(v + 1) * T], nl, False, True) for v in range(nvid)], 0)
        (yr * gg).sum().backward()
        errs = {"y": rel(y, yr), "dx": rel(xd.grad, xr.grad)}
        for n, t in mod.named_parameters():
            errs[n] = rel(t.grad, P[n].grad)
        bad = {k: f"{v:.1e}" for k, v in errs.items() if v > 1e-4}
        print(f"T={T} nvid={nvid} nl={nl} fused={fused}: max {max(errs.values()):.1e} bad {bad}", flush=True)
