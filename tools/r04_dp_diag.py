"""Round-4 diagnostic: where the N=1 RCCL bucket schedule's overhead goes (bench dp_schedule).

World-size-1 nccl group; bench's T=4096 2-video step with DataParallel(force_buckets=True) on and off,
host time spent issuing collectives per step, bucket sizes / offsets, and a variant whose collectives
are issued from a helper thread.
"""
import os
import socket
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import bench  # noqa: E402


def main():
    from factmx.dp import DataParallel
    from factmx.utils.runtime import freeze_host_heap
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    cfg, D, C, T, nv, clip, _ = bench.workload("havid")
    net, _ = bench.build_model(cfg, D, C, dev, seed=0, clip=clip)
    net.train()
    dp = DataParallel(net, broadcast=False, force_buckets=True)
    base = dp.flat.data_ptr()
    for k, bl in sorted(dp.block_buckets.items()):
        print("block", k, [((b.data_ptr() - base) // 4, b.numel()) for b in bl])
    print("rest", [((b.data_ptr() - base) // 4, b.numel()) for b in dp.rest_buckets], "total", dp.flat.numel())
    seqs, labels = [], []
    for s in range(1, nv + 1):
        f, l_ = bench.make_video(T, D, C, cfg, seed=s)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))
    fin = [0.0]

    def step():
        dp.zero_grad()
        loss, _ = net(seqs, labels, compute_loss=True)
        loss.backward()
        t0 = time.perf_counter()
        dp.finish_gradients()
        fin[0] += time.perf_counter() - t0

    def timed(active, k=20, thread=False):
        dp.active = active
        dp.issue_thread = thread
        step()
        torch.cuda.synchronize()
        dp.host_issue_s = 0.0
        fin[0] = 0.0
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / k, 1e3 * dp.host_issue_s / k, 1e3 * fin[0] / k

    for _ in range(3):
        step()
    freeze_host_heap()
    res = {"plain": [], "forced": [], "forced_thread": []}
    for _ in range(4):
        res["plain"].append(timed(False))
        res["forced"].append(timed(True))
        res["forced_thread"].append(timed(True, thread=True))
    for k, v in res.items():
        print(k, "ms/step, host issue ms/step, finish ms/step:", [tuple(round(x, 3) for x in t) for t in v])
        print("  median step", round(statistics.median(t[0] for t in v), 3))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
