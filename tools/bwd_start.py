"""Diagnostic: where the time between loss.backward() and the first factmx backward function goes
(engine start, the root node, the loss node).  python tools/bwd_start.py"""
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
    from factmx.models import vloss
    dp = DataParallel(net)
    seqs, labs = [], []
    for v in range(2):
        f, l_ = bench.make_video(4096, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))
    T = {}
    orig = vloss._LossFn.backward

    def lb(ctx, g):
        T["loss_enter"] = time.perf_counter()
        r = orig(ctx, g)
        T["loss_exit"] = time.perf_counter()
        return r
    vloss._LossFn.backward = staticmethod(lb)
    import gc
    for it in range(8):
        if it == 4:
            gc.disable()
            print("gc disabled")
        dp.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        torch.cuda.synchronize()
        T.clear()
        loss.grad_fn.register_prehook(lambda g: T.__setitem__("root", time.perf_counter()))
        for nf, _ in loss.grad_fn.next_functions:
            if nf is not None:
                nf.register_prehook(lambda g: T.__setitem__("loss_node", time.perf_counter()))
        t0 = time.perf_counter()
        loss.backward()
        t1 = time.perf_counter()
        dp.finish_gradients()
        torch.cuda.synchronize()
        print(" ".join(f"{k}:{1e6 * (v - t0):.0f}us" for k, v in sorted(T.items(), key=lambda kv: kv[1])),
              f"backward-returned:{1e6 * (t1 - t0):.0f}us", type(loss.grad_fn).__name__)


if __name__ == "__main__":
    main()
