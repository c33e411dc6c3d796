"""Diagnostic: each autograd backward function of the bench step with its host time and the device
time of its launches (events recorded at entry / exit on its stream), and the device idle time right
before it (the gap between the previous function's last launch completing and this one's first event),
to find host-bound backward functions.  python tools/bwd_marks.py"""
import inspect
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

REC = []


def wrap_fn(cls):
    orig = cls.backward

    def bw(ctx, *g):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        r = orig(ctx, *g)
        t1 = time.perf_counter()
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        REC.append((cls.__name__, t0, t1, e0, e1))
        return r
    cls.backward = staticmethod(bw)


def main():
    from factmx import functional as fxf
    from factmx.models import vloss, basic, blocks
    for mod in (fxf, vloss, basic, blocks):
        for _, c in inspect.getmembers(mod, inspect.isclass):
            if issubclass(c, torch.autograd.Function) and c is not torch.autograd.Function and c.__module__ == mod.__name__:
                wrap_fn(c)
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
    for it in range(5):
        REC.clear()
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        e_fwd = torch.cuda.Event(enable_timing=True)
        e_fwd.record()
        h_fwd = time.perf_counter()
        loss.backward()
        dp.finish_gradients()
        torch.cuda.synchronize()
    prev_e, prev_h = e_fwd, h_fwd
    tot_idle = 0.0
    print(f"{'function':28s} {'host_us':>8s} {'gpu_us':>8s} {'idle_before_us':>14s} {'host_at':>8s} {'gpu_at':>8s}")
    for name, t0, t1, e0, e1 in REC:
        idle = prev_e.elapsed_time(e0) * 1e3
        print(f"{name:28s} {1e6 * (t1 - t0):8.1f} {e0.elapsed_time(e1) * 1e3:8.1f} {idle:14.1f} "
              f"{1e3 * (t0 - h_fwd):8.2f} {e_fwd.elapsed_time(e0):8.2f}")
        prev_e = e1
    print("backward device end (ms after forward end):", e_fwd.elapsed_time(prev_e))


if __name__ == "__main__":
    main()
