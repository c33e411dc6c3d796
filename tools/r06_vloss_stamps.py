"""Round-6 diagnostic: host time between the stamps of vloss.run (FX_VLOSS_TIMES=1) over bench steps."""
import collections
import os
import sys

os.environ["FX_VLOSS_TIMES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from factmx.models import vloss  # noqa: E402


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
    acc = collections.defaultdict(float)
    n = 0
    for i in range(15):
        vloss.RUN_TIMES.clear()
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()
        dp.finish_gradients()
        if i >= 5:
            t = vloss.RUN_TIMES
            for (a, ta), (b, tb) in zip(t, t[1:]):
                acc[f"{a} -> {b}"] += tb - ta
            n += 1
    torch.cuda.synchronize()
    for k, v in acc.items():
        print(f"{1e6 * v / n:8.1f} us  {k}")


if __name__ == "__main__":
    main()
