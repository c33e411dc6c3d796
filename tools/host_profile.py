"""Diagnostic: where the HOST time of a bench step goes (cProfile over a few steps; GPU work is async,
so blocking device syncs show up as time inside .item()/.cpu()/.tolist()/synchronize).

python tools/host_profile.py
"""
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


def main():
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    net, _ = bench.build_model(cfg, bench.D_IN, bench.NCLS, dev)
    net.train()
    from factmx.dp import FlatGradReducer
    from factmx.optim import FusedAdam
    red = FlatGradReducer(net.parameters())
    opt = FusedAdam(net.parameters(), lr=1e-4, max_grad_norm=10.0, grad_flat=red.flat)
    seqs, labs = [], []
    for v in range(2):
        f, l_ = bench.make_video(4096, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))

    def step():
        red.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    print(f"plain: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms/step")
    # host-only cost of the forward: time spent before the first sync point is hard to isolate, so
    # also time forward and backward separately with a sync in between
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        red.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        opt.step()
        torch.cuda.synchronize()
        print(f"fwd host {1e3 * (t1 - t0):.2f} (+drain {1e3 * (t2 - t1):.2f})  bwd host {1e3 * (t3 - t2):.2f} "
              f"(+drain {1e3 * (t4 - t3):.2f}) ms")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
