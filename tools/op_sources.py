"""Diagnostic: which Python lines launch the glue kernels (fill / copy / add / cat ...) in one bench step.

python tools/op_sources.py  -> per aten op: count per step and the factmx source lines that issued them
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402

_UNUSED = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::cat", "aten::mul",
       "aten::index", "aten::index_add_", "aten::sum", "aten::neg", "aten::clone", "aten::item",
       "aten::_local_scalar_dense", "aten::sub", "aten::div", "aten::nonzero", "aten::masked_select",
       "aten::_to_copy", "aten::zeros", "aten::zeros_like", "aten::ones", "aten::full")


def main():
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    dev = torch.device("cuda", 0)
    cfg = bench.make_cfg()
    net, _ = bench.build_model(cfg, bench.D_IN, bench.NCLS, dev)
    net.train()
    from factmx.dp import FlatGradReducer
    red = FlatGradReducer(net.parameters())
    opt = torch.optim.Adam(net.parameters(), lr=1e-4)
    seqs, labs = [], []
    for v in range(2):
        f, l_ = bench.make_video(4096, bench.D_IN, bench.NCLS, cfg, seed=1 + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labs.append(torch.from_numpy(l_).to(dev))

    def step():
        red.zero_grad()
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(net.parameters(), 10.0)
        opt.step()

    agg = collections.defaultdict(collections.Counter)

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket.__name__)
            on_gpu = any(isinstance(a, torch.Tensor) and a.is_cuda for a in args)
            if on_gpu and name not in ("view", "_unsafe_view", "as_strided", "t", "transpose", "unsqueeze",
                                       "squeeze", "select", "slice", "expand", "permute", "reshape",
                                       "empty", "empty_strided", "detach", "alias", "split", "unbind",
                                       "_reshape_alias", "split_with_sizes", "narrow"):
                fr = [f for f in traceback.extract_stack()[:-1] if "factmx" in f.filename or "bench.py" in f.filename
                      or "torch/optim" in f.filename or "clip_grad" in f.filename or "torch/autograd" in f.filename
                      or "torch/nn" in f.filename]
                where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[::-1][:3]) or "?"
                agg[name][where] += 1
            return func(*args, **(kwargs or {}))

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with Log():
        step()
        torch.cuda.synchronize()
    tot = collections.Counter({k: sum(v.values()) for k, v in agg.items()})
    print("total device ops:", sum(tot.values()))
    for op, n in tot.most_common():
        print(f"== {op}: {n}")
        for where, k in agg[op].most_common(14):
            print(f"   {k:5d}  {where}")


if __name__ == "__main__":
    main()
