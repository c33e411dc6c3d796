"""Where the headline step's torch-side launches come from: one step of bench.py's havid workload under
torch.profiler (with stacks), aten ops that launch device work counted per call site in factmx/.

    python tools/r05_torch_ops.py > gpurun_out/torch_ops.txt
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import bench  # noqa: E402


def main():
    from factmx import native
    from factmx.dp import DataParallel
    native.load()
    cfg, D, C, T, nv, clip, _ = bench.workload("havid")
    dev = torch.device("cuda", 0)
    net, _ = bench.build_model(cfg, D, C, dev, seed=0, clip=clip)
    net.train()
    dp = DataParallel(net)
    seqs, labels = [], []
    for s, Tv in zip(range(1, nv + 1), bench.video_lengths("havid", T, nv)):
        f, l_ = bench.make_video(Tv, D, C, cfg, seed=s)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))

    def step():
        dp.zero_grad()
        loss, _ = net(seqs, labels, compute_loss=True)
        loss.backward()
        dp.finish_gradients()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    keep = ("aten::copy_", "aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::cat", "aten::clamp",
            "aten::mul", "aten::sum", "aten::index", "aten::div", "aten::sub", "aten::where", "aten::clone",
            "aten::contiguous", "aten::stack", "aten::neg", "aten::max", "aten::exp", "aten::_to_copy",
            "aten::index_put_", "aten::gather", "aten::masked_fill", "aten::full")
    sites = collections.Counter()
    names = collections.Counter()
    for ev in prof.events():
        if ev.name not in keep:
            continue
        names[ev.name] += 1
        fr = [f for f in (ev.stack or []) if "factmx" in f or "bench" in f]
        if fr:
            site = " <- ".join(f.split("/")[-1] for f in fr[:3])
        else:
            par, up = [], ev.cpu_parent
            while up is not None and len(par) < 3:
                par.append(up.name[:60])
                up = up.cpu_parent
            site = "(engine) " + " <- ".join(par)
        sites[(ev.name, site)] += 1
    print("aten ops (calls per step):")
    for k, v in names.most_common():
        print(f"{v:5d} {k}")
    print("\nby call site:")
    for (n, s), v in sites.most_common(80):
        print(f"{v:5d} {n:22s} {s}")


if __name__ == "__main__":
    main()
