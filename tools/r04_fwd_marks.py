"""Round-4 diagnostic: host time vs device time at marks inside one bench step (block entries/exits,
segmentation, the loss phase, backward), to see which stretches are host-issue bound; then a cProfile
of a few steps (host self time per function).  python tools/r04_fwd_marks.py"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

MARKS = []


def mark(name):
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    MARKS.append((name, time.perf_counter(), e))


def wrap(obj, attr, name):
    fn = getattr(obj, attr)

    def w(*a, **k):
        mark(name + ">")
        r = fn(*a, **k)
        mark(name + "<")
        return r
    setattr(obj, attr, w)


def wrap_bwd(cls, name):
    fn = cls.backward

    def w(ctx, *a):
        mark(name + ".bwd>")
        r = fn(ctx, *a)
        mark(name + ".bwd<")
        return r
    cls.backward = staticmethod(w)


def main():
    from factmx.dp import DataParallel
    from factmx.models import blocks, vloss
    from factmx import functional as fxf
    from factmx.utils.runtime import freeze_host_heap
    cfg, D, C, Tn, nv, clip, _ = bench.workload("havid")
    dev = torch.device("cuda", 0)
    net, _ = bench.build_model(cfg, D, C, dev, seed=0, clip=clip)
    net.train()
    dp = DataParallel(net)
    seqs, labels = [], []
    for s in range(1, nv + 1):
        f, l_ = bench.make_video(Tn, D, C, cfg, seed=s)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))

    def step():
        dp.zero_grad()
        mark("start")
        loss, _ = net(seqs, labels, compute_loss=True)
        mark("fwd_end")
        loss.backward()
        mark("bwd_issued")
        dp.finish_gradients()
        mark("end")

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    freeze_host_heap()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(6):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(45)
    for name in dir(blocks):
        cls = getattr(blocks, name)
        if isinstance(cls, type) and hasattr(cls, "forward_batch"):
            wrap(cls, "forward_batch", name)
    for mod, attr in ((vloss, "run"), (vloss, "resolve_pending"), (fxf, "resolve_backward_status"),
                      (blocks, "_label_to_host")):
        if hasattr(mod, attr):
            wrap(mod, attr, attr)
    for name in ("segments_from_probs_batched", "segments_from_probs", "mstcn", "decoder", "x2y", "gru_bidir"):
        if hasattr(fxf, name):
            wrap(fxf, name, name)
    import threading
    for name in dir(fxf):
        cls = getattr(fxf, name)
        if isinstance(cls, type) and issubclass(cls, torch.autograd.Function) and "backward" in cls.__dict__:
            wrap_bwd(cls, name)
    wrap_bwd(vloss._LossFn, "_LossFn")
    for _ in range(2):
        MARKS.clear()
        step()
        torch.cuda.synchronize()
    if vloss.RUN_TIMES:
        t = vloss.RUN_TIMES[-15:]
        for (a, ta), (b, tb) in zip(t, t[1:]):
            print(f"run: {a:>12s} -> {b:12s} {1e6 * (tb - ta):8.1f} us")
    h0, e0 = MARKS[0][1], MARKS[0][2]
    ph, pg = 0.0, 0.0
    for name, h, e in MARKS:
        hh, gg = 1e3 * (h - h0), e0.elapsed_time(e)
        print(f"{name:34s} host {hh:8.3f} (+{hh - ph:6.3f})  gpu {gg:8.3f} (+{gg - pg:6.3f})  lead {gg - hh:7.3f}")
        ph, pg = hh, gg


if __name__ == "__main__":
    main()
