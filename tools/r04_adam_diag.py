"""Round-4 diagnostic: why is bench's train_step_with_adam leg slower than the fixed-weight step?

Runs the bench workload, then N Adam steps, recording per step: wall ms (sync each step), the TDU
segment counts, and the torch allocator's cudaMalloc count / reserved bytes.  Also times a block of
Adam steps without per-step syncs, and the same number of fixed-weight steps, for comparison.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import torch  # noqa: E402
import bench  # noqa: E402


GC = []


def _gc_cb(phase, info):
    if phase == "start":
        GC.append([info["generation"], time.perf_counter(), None, 0])
    elif GC:
        GC[-1][2] = time.perf_counter()
        GC[-1][3] = info.get("collected", 0)


def gc_report(tag):
    big = [(g, round(1e3 * (b - a), 2), c) for g, a, b, c in GC if b is not None and (g == 2 or b - a > 1e-3)]
    n = [sum(1 for x in GC if x[0] == g) for g in range(3)]
    print(f"  gc during {tag}: collections per generation {n}, slow/gen2 ones (gen, ms, collected) {big}", flush=True)
    GC.clear()


def main():
    import gc
    gc.callbacks.append(_gc_cb)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from factmx.dp import DataParallel
    from factmx.optim import FusedAdam
    cfg, D, C, T, nv, clip, _ = bench.workload("havid")
    dev = torch.device("cuda", 0)
    net, _ = bench.build_model(cfg, D, C, dev, seed=0, clip=clip)
    net.train()
    dp = DataParallel(net)
    seqs, labels = [], []
    for s in range(1, nv + 1):
        f, l_ = bench.make_video(T, D, C, cfg, seed=s)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))

    def step():
        dp.zero_grad()
        loss, _ = net(seqs, labels, compute_loss=True)
        loss.backward()
        dp.finish_gradients()

    def timed(fn, k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / k

    for _ in range(5):
        step()
    gc_report("warmup")
    print("fixed  ms/step", round(timed(step, n), 3), "S", bench.video_segments(net), flush=True)
    gc_report("fixed")
    w0 = [p.detach().clone() for p in net.parameters()]
    opt = FusedAdam(net.parameters(), lr=cfg.lr, max_grad_norm=cfg.clip_grad_norm, grad_flat=dp.flat)

    def astep():
        step()
        opt.step()
    astep()
    st = torch.cuda.memory_stats()
    m0 = st.get("num_alloc_retries", 0), torch.cuda.memory_reserved()
    gc_report("adam first")
    print("adam   ms/step", round(timed(astep, n), 3), "S", bench.video_segments(net), flush=True)
    gc_report("adam block")
    for i in range(n):
        a0 = torch.cuda.memory_stats().get("num_device_alloc", 0)
        ms = timed(astep, 1)
        a1 = torch.cuda.memory_stats().get("num_device_alloc", 0)
        gc_report(f"step {i}")
        print(f"adam step {i}: {ms:.3f} ms S {bench.video_segments(net)} device_allocs +{a1 - a0} "
              f"reserved {torch.cuda.memory_reserved() / 2**20:.0f} MiB", flush=True)
    print("alloc retries / reserved at start", m0, flush=True)
    # the same weights frozen at the drifted point: fixed-weight steps there
    print("fixed at drifted weights ms/step", round(timed(step, n), 3), "S", bench.video_segments(net), flush=True)
    with torch.no_grad():
        for p_, w in zip(net.parameters(), w0):
            p_.copy_(w)
    print("fixed again ms/step", round(timed(step, n), 3), "S", bench.video_segments(net), flush=True)
    gc_report("fixed again")
    gc.freeze()
    print("after gc.freeze(): fixed ms/step", round(timed(step, n), 3), flush=True)
    gc_report("fixed frozen")
    print("after gc.freeze(): adam ms/step", round(timed(astep, n), 3), flush=True)
    gc_report("adam frozen")


if __name__ == "__main__":
    main()
