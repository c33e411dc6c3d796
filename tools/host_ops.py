"""Diagnostic: host (CPU) time per autograd node / op of the bench step (torch.profiler, CPU activity
only), so the Python backward functions that leave the GPU idle can be found.

python tools/host_ops.py
"""
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

    def step():
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()
        dp.finish_gradients()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    print(f"step {(time.perf_counter() - t0) / 10 * 1e3:.2f} ms", flush=True)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(3):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=45))


if __name__ == "__main__":
    main()
