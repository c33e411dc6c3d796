"""Diagnostic: autograd start-up latency (loss.backward() -> first Function.backward) for graphs shaped
like the bench step (44 chained custom Functions, 415 parameters), with / without .grad views of a flat
buffer and with / without tensors saved for backward.  python tools/ag_probe.py"""
import time

import torch


class F(torch.autograd.Function):
    first = [None]

    @staticmethod
    def forward(ctx, x, *ps):
        if F.save:
            ctx.save_for_backward(x, *ps)
        return x * 2

    @staticmethod
    def backward(ctx, g):
        if F.first[0] is None:
            F.first[0] = time.perf_counter()
        return (g * 2,) + (None,) * (len(ctx.needs_input_grad) - 1)


def run(nfn, nparam, flat_views, save):
    F.save = save
    ps = [torch.zeros(256, device="cuda", requires_grad=True) for _ in range(nparam)]
    if flat_views:
        flat = torch.zeros(256 * nparam, device="cuda")
        for i, p in enumerate(ps):
            p.grad = flat[256 * i:256 * (i + 1)]
    per = max(1, nparam // nfn)
    best = 1e9
    for _ in range(20):
        x = torch.randn(1024, device="cuda", requires_grad=True)
        y = x
        for k in range(nfn):
            y = F.apply(y, *ps[k * per:(k + 1) * per])
        loss = y.sum()
        torch.cuda.synchronize()
        F.first[0] = None
        t0 = time.perf_counter()
        loss.backward()
        best = min(best, F.first[0] - t0)
        torch.cuda.synchronize()
    print(f"fns {nfn:3d} params {nparam:4d} flat_views {flat_views} save {save}: start {best * 1e6:7.1f} us")


for args in [(1, 415, False, False), (44, 415, False, False), (44, 415, True, False), (44, 415, True, True),
             (44, 0, False, True)]:
    run(*args)
