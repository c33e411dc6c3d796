"""Round-4 diagnostic: which objects of a bench step end up in reference cycles (cyclic garbage that
only a full gc pass frees -- a 60 ms gen-2 collection every few dozen steps)."""
import collections
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import torch  # noqa: E402
import bench  # noqa: E402


def describe(o):
    t = type(o)
    name = f"{t.__module__}.{t.__qualname__}"
    if isinstance(o, dict):
        keys = list(o.keys())[:6]
        name += f" keys={keys}"
    elif callable(o) and hasattr(o, "__qualname__"):
        name += f" {o.__qualname__}"
    elif hasattr(o, "__dict__") and not isinstance(o, type):
        name += f" attrs={list(vars(o))[:6]}"
    return name


def main():
    from factmx.dp import DataParallel
    cfg, D, C, T, nv, clip, _ = bench.workload(sys.argv[1] if len(sys.argv) > 1 else "havid")
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
    gc.collect()
    gc.set_debug(gc.DEBUG_SAVEALL)
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    n = gc.collect()
    garbage = list(gc.garbage)
    gc.set_debug(0)
    print(f"cyclic garbage of 2 steps: {n} objects", flush=True)
    cnt = collections.Counter(describe(o) for o in garbage)
    for k, v in cnt.most_common(60):
        print(f"{v:6d}  {k}")
    ids = {id(o) for o in garbage}
    # a few cycles spelled out: follow referents inside the garbage set
    shown = 0
    for o in garbage:
        if shown >= 8:
            break
        if not (hasattr(o, "__dict__") and not isinstance(o, type)) and not callable(o):
            continue
        chain, cur, seen = [describe(o)], o, {id(o)}
        for _ in range(8):
            nxt = [r for r in gc.get_referents(cur) if id(r) in ids]
            if not nxt:
                break
            cur = nxt[0]
            if id(cur) in seen:
                chain.append("<back to " + describe(cur)[:60] + ">")
                break
            seen.add(id(cur))
            chain.append(describe(cur)[:100])
        print("CHAIN:", " -> ".join(chain), flush=True)
        shown += 1


if __name__ == "__main__":
    main()
