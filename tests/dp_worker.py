"""One rank of the GPU data-parallel test (tests/test_gpu_dp.py); started as a child process.

Every rank runs the real FACT_CLIP lockstep step (bench.py's HAViD-holdout model, ``--videos``
seg10 videos of T frames on its own shard of the global batch) through factmx.dp.DataParallel on
cuda:0 over the gloo backend (two ranks share the one leased GPU; RCCL refuses two ranks on one
device), then writes what the test checks: the reduced flat gradient, the order in which block
buckets launched from the backward hooks, and a checksum of its weights after the rank-0 broadcast.
Rank 1 builds its model from another seed, so identical weights prove the broadcast.

Reference semantics being parallelised: per-video loss averaging, blocks.py:913-915.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--T", type=int, default=2048)
    ap.add_argument("--videos", type=int, default=2)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    import bench
    from factmx.dp import DataParallel
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = bench.make_cfg()
        D, C = bench.D_IN, bench.NCLS
        net, _ = bench.build_model(cfg, D, C, dev, seed=rank)       # rank 1: other weights until broadcast
        net.train()
        dp = DataParallel(net)
        wsum = torch.cat([p.detach().reshape(-1).double() for p in net.parameters()])
        seeds = [1 + rank * args.videos + v for v in range(args.videos)]
        vids = [bench.make_video(args.T, D, C, cfg, seed=s) for s in seeds]
        seqs = [torch.from_numpy(f).to(dev) for f, _ in vids]
        labs = [torch.from_numpy(l_).to(dev) for _, l_ in vids]
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()
        # a block part (k, name) as -1 - k
        early = [k if isinstance(k, int) else -1 - k[0] for k in dp.hook_launched]
        dp.finish_gradients()
        torch.cuda.synchronize()
        np.savez(os.path.join(args.out, f"rank{rank}.npz"), flat=dp.flat.detach().cpu().numpy(),
                 early=np.asarray(early, dtype=np.int64), nblk=np.int64(len(net.block_list)),
                 tail=np.int64(dp.tail_bytes),
                 wsum=np.asarray([float(wsum.sum()), float((wsum * wsum).sum())]),
                 loss=np.float64(loss.item()), S=np.asarray(bench.video_segments(net), dtype=np.int64))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
