"""Round-6 diagnostic: host time per autograd Function (forward and backward, the backward ones run on the
autograd device thread, which cProfile of the main thread does not see) and per block / loss-phase entry point,
over a few bench steps.  python tools/r06_host_ops.py"""
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

ACC = collections.defaultdict(lambda: [0.0, 0])


def timed(name, fn):
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            e = ACC[name]
            e[0] += time.perf_counter() - t0
            e[1] += 1
    return w


def patch():
    from factmx import functional as fxf
    from factmx.models import blocks, vloss
    for mod in (fxf, vloss):
        for n in dir(mod):
            c = getattr(mod, n)
            if isinstance(c, type) and issubclass(c, torch.autograd.Function) and c is not torch.autograd.Function:
                for ph in ("forward", "backward"):
                    if ph in c.__dict__:
                        setattr(c, ph, staticmethod(timed(f"{n}.{ph}", c.__dict__[ph].__func__)))
    for cls in (blocks.InputBlock, blocks.UpdateBlock, blocks.UpdateBlockTDU):
        cls.forward_batch = timed(cls.__name__ + ".forward_batch", cls.forward_batch)
    vloss.run = timed("vloss.run", vloss.run)
    vloss.EarlyMatch.__call__ = timed("EarlyMatch.__call__", vloss.EarlyMatch.__call__)
    vloss.EarlyMatch.matches = timed("EarlyMatch.matches", vloss.EarlyMatch.matches)
    fxf.segments_from_probs_batched = timed("segments_from_probs_batched", fxf.segments_from_probs_batched)


def main():
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    net, _ = bench.build_model(cfg, bench.D_IN, bench.NCLS, dev)
    net.train()
    from factmx.dp import DataParallel
    dp = DataParallel(net)
    seqs, labs = [], []
    for v in range(2):
        f, l_ = bench.make_video(4096, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))

    def step():
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()
        dp.finish_gradients()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    patch()
    n = 10
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    ACC.clear()
    t0 = time.perf_counter()
    tf = tb = 0.0
    for _ in range(n):
        a = time.perf_counter()
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        b = time.perf_counter()
        loss.backward()
        dp.finish_gradients()
        c = time.perf_counter()
        tf += b - a
        tb += c - b
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"{1e3 * el / n:.2f} ms/step; host in forward call {1e3 * tf / n:.2f} ms, in backward call {1e3 * tb / n:.2f} ms")
    for k, (t, c) in sorted(ACC.items(), key=lambda kv: -kv[1][0]):
        print(f"  {1e3 * t / n:8.3f} ms/step  {c / n:6.1f} calls/step  {1e6 * t / max(c, 1):8.1f} us/call  {k}")
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
