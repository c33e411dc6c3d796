"""World-size-1 RCCL run of the data-parallel schedule (tests/test_gpu_rccl.py); a child process.

Opens a one-rank ``nccl`` (= RCCL on ROCm) process group on cuda:0 and runs bench.py's FACT_CLIP
lockstep step (HAViD-holdout dims, ``--videos`` seg10 videos of T frames) through
factmx.dp.DataParallel twice: with the per-block bucket schedule switched off (the plain step) and
forced on (``force_buckets=True``: hooks, the collective stream waiting on the compute and side
streams, one RCCL all-reduce (AVG) per bucket).  The AVG over one rank is the identity, so the two
flat gradients must be bitwise equal.  It also times both schedules (alternating rounds) and writes
the overhead.  Reference semantics: the per-video loss mean of blocks.py:913-915.
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--T", type=int, default=4096)
    ap.add_argument("--videos", type=int, default=2)
    ap.add_argument("--time-steps", type=int, default=10)
    args = ap.parse_args()
    import bench
    from factmx.dp import DataParallel
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        cfg = bench.make_cfg()
        D, C = bench.D_IN, bench.NCLS
        net, _ = bench.build_model(cfg, D, C, dev, seed=0)
        net.train()
        dp = DataParallel(net, force_buckets=True)
        vids = [bench.make_video(args.T, D, C, cfg, seed=s) for s in range(1, 1 + args.videos)]
        seqs = [torch.from_numpy(f).to(dev) for f, _ in vids]
        labs = [torch.from_numpy(l_).to(dev) for _, l_ in vids]

        def step():
            dp.zero_grad()
            loss, _ = net(seqs, labs, compute_loss=True)
            loss.backward()
            dp.finish_gradients()
            return loss

        def run(active):
            dp.active = active
            loss = step()
            torch.cuda.synchronize()
            # (a block part (k, name) as -1 - k)
            return (dp.flat.detach().cpu().numpy().copy(), float(loss.item()),
                    [k if isinstance(k, int) else -1 - k[0] for k in dp.hook_launched])

        run(False)                         # warm-up (allocator, matching caches)
        plain1, loss1, _ = run(False)
        plain2, loss2, _ = run(False)
        forced, loss3, early = run(True)

        def timed(active, k):
            dp.active = active
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(k):
                step()
            torch.cuda.synchronize()
            return 1e3 * (time.perf_counter() - t0) / k

        plain_ms, forced_ms = [], []
        for _ in range(3):
            plain_ms.append(timed(False, args.time_steps))
            forced_ms.append(timed(True, args.time_steps))
        np.savez(os.path.join(args.out, "rccl.npz"), plain1=plain1, plain2=plain2, forced=forced,
                 early=np.asarray(early, dtype=np.int64), nblk=np.int64(len(net.block_list)),
                 tail=np.int64(dp.tail_bytes),
                 loss=np.asarray([loss1, loss2, loss3]))
        with open(os.path.join(args.out, "rccl.json"), "w") as f:
            json.dump(dict(plain_ms=plain_ms, forced_ms=forced_ms, backend=dist.get_backend(),
                           S=bench.video_segments(net)), f)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
