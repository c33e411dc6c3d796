"""Diagnostic: where does one bench step spend its time (host vs device, per stage)?

python tools/step_profile.py [--T 4096] [--videos 2]
Prints synchronised stage timings and the torch.profiler top host-time ops.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=4096)
    ap.add_argument("--videos", type=int, default=2)
    ap.add_argument("--trace", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    net, _ = bench.build_model(cfg, bench.D_IN, bench.NCLS, dev)
    net.train()
    from factmx.dp import FlatGradReducer
    red = FlatGradReducer(net.parameters())
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    seqs, labs = [], []
    for v in range(args.videos):
        f, l_ = bench.make_video(args.T, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))

    def sync():
        torch.cuda.synchronize()
        return time.perf_counter()

    def step(timed=False):
        t = [sync()]
        red.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        t.append(sync())
        loss.backward()
        t.append(sync())
        torch.nn.utils.clip_grad_norm_(net.parameters(), 10.0)
        opt.step()
        t.append(sync())
        if timed:
            print(f"fwd+loss {1e3*(t[1]-t[0]):.1f} ms  bwd {1e3*(t[2]-t[1]):.1f} ms  opt {1e3*(t[3]-t[2]):.1f} ms",
                  flush=True)

    for _ in range(3):
        step()
    for _ in range(3):
        step(timed=True)

    # per-block forward timing (one video)
    blocks = net.block_list
    orig = [b.forward for b in blocks]
    times = {}

    def wrap(i, fn):
        def f(*a, **k):
            t0 = sync()
            r = fn(*a, **k)
            times.setdefault(i, []).append(sync() - t0)
            return r
        return f
    for i, b in enumerate(blocks):
        b.forward = wrap(i, orig[i])
    loss, _ = net(seqs[:1], labs[:1], compute_loss=True)
    t0 = sync()
    loss.backward()
    tb = sync() - t0
    for i, b in enumerate(blocks):
        b.forward = orig[i]
    print("per-block fwd ms (1 video):", {i: round(1e3 * sum(v), 2) for i, v in times.items()}, "bwd", round(1e3 * tb, 1))

    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        step()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=30, max_name_column_width=60))
    if args.trace:
        prof.export_chrome_trace(os.path.join(ROOT, "gpurun_out", "step_trace.json"))


if __name__ == "__main__":
    main()
