"""Diagnostic: host time of each phase of the bench step (zero_grad / forward / backward / finish / the
return to the caller) next to when the GPU reaches the same points (events), to find where the GPU waits
for the host.  python tools/phase_times.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


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
    names = ["start", "zero_grad", "forward", "backward", "finish", "return"]

    def step(rec):
        ev = [torch.cuda.Event(enable_timing=True) for _ in names]
        t = [time.perf_counter()]
        ev[0].record()
        dp.zero_grad()
        t.append(time.perf_counter()); ev[1].record()
        loss, _ = net(seqs, labs, compute_loss=True)
        t.append(time.perf_counter()); ev[2].record()
        loss.backward()
        t.append(time.perf_counter()); ev[3].record()
        dp.finish_gradients()
        t.append(time.perf_counter()); ev[4].record()
        del loss
        t.append(time.perf_counter()); ev[5].record()
        rec.append((t, ev))

    recs = []
    for _ in range(3):
        step([])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        step(recs)
    torch.cuda.synchronize()
    print(f"{(time.perf_counter() - t0) / 8 * 1e3:.2f} ms/step")
    base_h, base_e = recs[0][0][0], recs[0][1][0]
    for t, ev in recs:
        hs = "  ".join(f"{n}:{1e3 * (x - base_h):7.2f}" for n, x in zip(names, t))
        gs = "  ".join(f"{base_e.elapsed_time(e):7.2f}" for e in ev)
        print("host", hs)
        print(" gpu", gs)


if __name__ == "__main__":
    main()
