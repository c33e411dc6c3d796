"""Round-4 diagnostic: which host call at the start of the forward waits for the device (the GPU idles
~0.7 ms at every step boundary while the host is ~4.7 ms ahead at zero_grad).  Wraps the forward's
first calls with host timers for a few bench steps."""
import functools
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import torch  # noqa: E402
import bench  # noqa: E402

T = {}


def timed(mod, name):
    f = getattr(mod, name)

    @functools.wraps(f)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            T.setdefault(name, []).append(1e3 * (time.perf_counter() - t0))
    setattr(mod, name, w)


def main():
    from factmx.dp import DataParallel
    from factmx.models import blocks, vloss
    from factmx import functional as fxf
    cfg, D, C, Tn, nv, clip, _ = bench.workload("havid")
    dev = torch.device("cuda", 0)
    net, _ = bench.build_model(cfg, D, C, dev, seed=0, clip=clip)
    net.train()
    dp = DataParallel(net)
    seqs, labels = [], []
    for s in range(1, nv + 1):
        f, l_ = bench.make_video(Tn, D, C, cfg, seed=s)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))
    for mod, name in ((vloss, "resolve_pending"), (blocks, "_label_to_host"), (blocks, "_batchable"),
                      (vloss, "EarlyMatch"), (fxf, "resolve_backward_status")):
        timed(mod, name)
    orig_fb = type(net)._forward_batch

    def fb(self, *a, **k):
        T.setdefault("_forward_batch_entry", []).append(1e3 * (time.perf_counter() - T["_t_step"]))
        return orig_fb(self, *a, **k)
    type(net)._forward_batch = fb

    def step():
        T["_t_step"] = time.perf_counter()
        dp.zero_grad()
        loss, _ = net(seqs, labels, compute_loss=True)
        T.setdefault("forward_total", []).append(1e3 * (time.perf_counter() - T["_t_step"]))
        loss.backward()
        dp.finish_gradients()

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    for k in list(T):
        if not k.startswith("_t"):
            T[k] = []
    for _ in range(6):
        step()
    torch.cuda.synchronize()
    for k, v in T.items():
        if not k.startswith("_t"):
            print(f"{k:28s} " + " ".join(f"{x:7.3f}" for x in v), flush=True)


if __name__ == "__main__":
    main()
