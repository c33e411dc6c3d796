"""Diagnostic: node types of the bench step's autograd graph (the engine's start-up cost grows with it).
python tools/graph_nodes.py"""
import collections
import os
import sys

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
    seqs, labs = [], []
    for v in range(2):
        f, l_ = bench.make_video(4096, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))
    loss, _ = net(seqs, labs, compute_loss=True)
    seen, cnt, stack = set(), collections.Counter(), [loss.grad_fn]
    while stack:
        fn = stack.pop()
        if fn is None or fn in seen:
            continue
        seen.add(fn)
        cnt[type(fn).__name__] += 1
        for nf, _ in fn.next_functions:
            stack.append(nf)
    print("nodes", len(seen))
    for k, v in cnt.most_common(40):
        print(f"{v:5d} {k}")


if __name__ == "__main__":
    main()
