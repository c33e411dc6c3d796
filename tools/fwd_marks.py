"""Diagnostic: host time vs device time at marks inside the forward (block entries/exits, the loss
phase), to see which stretches of the forward are host-issue bound.  python tools/fwd_marks.py"""
import os
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


def main():
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    net, _ = bench.build_model(cfg, bench.D_IN, bench.NCLS, dev)
    net.train()
    from factmx.dp import DataParallel
    from factmx.models import blocks, vloss
    from factmx import functional as fxf
    dp = DataParallel(net)
    for cls in (blocks.InputBlock, blocks.UpdateBlock, blocks.UpdateBlockTDU):
        wrap(cls, "forward_batch", cls.__name__)
    wrap(vloss, "run", "loss.run")
    wrap(vloss.EarlyMatch, "__call__", "match.launch")
    wrap(vloss.EarlyMatch, "matches", "hungarian")
    wrap(fxf, "segments_from_probs_batched", "segments")
    seqs, labs = [], []
    for v in range(2):
        f, l_ = bench.make_video(4096, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))
    for it in range(6):
        MARKS.clear()
        dp.zero_grad()
        mark("start")
        loss, _ = net(seqs, labs, compute_loss=True)
        mark("fwd_end")
        loss.backward()
        mark("bwd_issued")
        dp.finish_gradients()
        torch.cuda.synchronize()
        mark("end")
        torch.cuda.synchronize()
    h0, e0 = MARKS[0][1], MARKS[0][2]
    for name, h, e in MARKS:
        print(f"{name:24s} host {1e3 * (h - h0):8.3f}  gpu {e0.elapsed_time(e):8.3f}")


if __name__ == "__main__":
    main()
