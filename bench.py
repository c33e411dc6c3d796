#!/usr/bin/env python
"""Benchmark: FACT_CLIP forward+loss+backward(+grad all-reduce)+clip+Adam frames/s on MI355X.

Workload (BASELINE.json metric, SURVEY.md section 8d "primary"): FACT_CLIP with
the HAViD view0_lh_pt_holdout dims and FACT.ntoken 32 (H=512, A=F=256, FF=512,
8 heads, 10 TCN layers, blocks iuUU), D=2048, C=75, T=4096 frames per video,
synthetic "seg10" videos (10 ground-truth segments, piecewise-constant
features), random-init weights (torch.manual_seed), fp32 parity arithmetic,
dropout / channel masking / time mask off (as in the reference CPU baseline).
One step = the reference train step (scripts/train.py:262-268) over
``--videos`` videos per rank: zero_grad, forward + loss, backward, gradient
all-reduce (N>1), clip_grad_norm_(10), Adam(lr 1e-4).

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Rank 0 prints one JSON line.  ``value`` = all frames processed by all ranks /
max-over-ranks wall time of the K timed steps.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

DOMINANT_KERNEL = "gemm_f32_wide8_kernel<1, 0>"   # rocprofv3 name: fx::(anonymous namespace)::gemm_f32_wide8_kernel<1, 0>
METRIC = "frames/sec FACT_CLIP fwd+bwd, T=4096 D=2048 Nact=32, at 1/2/4/8 GPUs"
F32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HOLDOUT = [51, 53, 61, 67, 56]   # havid_view0_lh_pt_holdout.yaml
D_IN, NCLS, NTOKEN, T_DEFAULT = 2048, 75, 32, 4096


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_cfg(ntoken=NTOKEN):
    """HAViD view0_lh_pt holdout dims (the reference yaml) with FACT.ntoken 32, dropout off."""
    from factmx.configs import get_cfg_defaults
    cfg = get_cfg_defaults()
    cfg.Bi.update(dict(hid_dim=512, dropout=0.0, a="sca", a_nhead=8, a_ffdim=512, a_layers=6, a_dim=256,
                       f="m", f_layers=10, f_ln=False, f_dim=256, f_ngp=1))
    for blk in (cfg.Bu, cfg.BU):
        blk.update(dict(a="sa", a_dim=None, a_ffdim=None, a_layers=1, a_nhead=8, dropout=None, f=None,
                        f_dim=None, f_layers=10, f_ln=None, f_ngp=None, hid_dim=None))
    cfg.BU.s_layers = 1
    cfg.FACT.update(dict(block="iuUU", cmr=0.0, fpos=False, mwt=0.1, ntoken=ntoken, trans=False))
    cfg.Loss.update(dict(a2fc=1.0, bgw=1.0, match="o2o", pc=0.2, sw=5.0))
    cfg.Loss.nullw = ntoken / ((ntoken - 10) * NCLS)      # train_tools.py:54-71, avg transcript length 10
    cfg.TM.use = False
    cfg.CLIP.update(dict(temp=0.1, contrastive_weight=0.5, fact_loss_weight=0.5, projection_hidden_dim=512,
                         projection_dropout=0.0))
    cfg.holdout_mode = True
    cfg.holdout_classes = list(HOLDOUT)
    cfg.use_clip = True
    cfg.batch_size = 2
    cfg.lr = 1e-4
    cfg.optimizer = "Adam"
    cfg.clip_grad_norm = 10.0
    return cfg


def make_video(T, D, C, cfg, seed, nseg=10):
    """seg10 synthetic video: 10 segments with sorted random cut points,
    one randn(D) prototype per segment, labels seen[(7i+3) % |seen|]."""
    g = torch.Generator().manual_seed(seed)
    seen = [c for c in range(C) if c not in set(cfg.holdout_classes)]
    cuts = torch.sort(torch.randperm(T - 1, generator=g)[: nseg - 1] + 1).values.tolist()
    bounds = [0] + cuts + [T]
    protos = torch.randn(nseg, D, generator=g)
    feats = torch.empty(T, D)
    label = torch.empty(T, dtype=torch.int64)
    for i in range(nseg):
        feats[bounds[i]:bounds[i + 1]] = protos[i]
        label[bounds[i]:bounds[i + 1]] = seen[(7 * i + 3) % len(seen)]
    return feats.numpy(), label.numpy()


def text_embeddings(C):
    g = torch.Generator().manual_seed(0)
    t = torch.randn(C, 512, generator=g)
    return t / t.norm(dim=1, keepdim=True)


def build_model(cfg, D, C, device, seed=0):
    from factmx.models.blocks import FACT_CLIP
    from factmx.models.loss import MatchCriterion
    text = text_embeddings(C)
    torch.manual_seed(seed)
    net = FACT_CLIP(cfg, D, C, text_embeddings=text.clone())
    net.mcriterion = MatchCriterion(cfg, C, [])
    return net.to(device), text


def traffic_from_profiles(kernel_prefix):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(ROOT, "profiles", "pmc_dominant.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            d = json.load(f)
        if kernel_prefix in str(d.get("kernel", "")):
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(T, min_seconds=10.0, min_steps=2):
    """The CPU oracle (fp32 PyTorch restatement pinned to the reference) timed on host cores:
    one video per step, full T, forward+loss+backward+Adam, repeated until >= min_seconds of
    CPU work (bounded sample, ~10 s); also counts algorithmic FLOPs."""
    from torch.utils.flop_counter import FlopCounterMode
    from oracle import fact_oracle as fo
    cfg = make_cfg()
    net, text = build_model(cfg, D_IN, NCLS, "cpu", seed=0)
    spec = fo.resolve_spec(cfg, D_IN, NCLS, clip=True)
    P = {n: p.detach().clone().float().requires_grad_(True) for n, p in net.named_parameters()}
    opt = torch.optim.Adam(list(P.values()), lr=1e-4)
    feats, label = make_video(T, D_IN, NCLS, cfg, seed=1)
    seq = torch.from_numpy(feats)

    def step():
        for p in P.values():
            p.grad = None
        out = fo.forward(spec, P, seq)
        fo.predict(spec, out, text)
        total, _, _, _ = fo.video_loss(spec, out, label, text)
        total.backward()
        torch.nn.utils.clip_grad_norm_(list(P.values()), 10.0)
        opt.step()

    with FlopCounterMode(display=False) as fc:
        step()
    flops = fc.get_total_flops()
    t0 = time.perf_counter()
    videos_timed = 0
    while videos_timed < min_steps or time.perf_counter() - t0 < min_seconds:
        step()
        videos_timed += 1
    dt = time.perf_counter() - t0
    return dict(value=round(videos_timed * T / dt, 1), unit="frames/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{videos_timed} steps x 1 video (T={T}, seg10) fwd+loss+bwd+Adam, oracle fp32 "
                       f"(1 untimed warm-up step, {dt:.1f} s timed)"), flops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--videos", type=int, default=2, help="videos per rank per step (HAViD batch_size)")
    ap.add_argument("--T", type=int, default=T_DEFAULT)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from factmx import native
    from factmx.dp import FlatGradReducer
    from factmx.optim import FusedAdam
    lib = native.load()

    cfg = make_cfg()
    net, _ = build_model(cfg, D_IN, NCLS, dev, seed=0)
    net.train()
    reducer = FlatGradReducer(net.parameters())
    # clip_grad_norm_(cfg.clip_grad_norm) + Adam(lr) of scripts/train.py:265-267, fused on the flat buffers
    opt = FusedAdam(net.parameters(), lr=cfg.lr, max_grad_norm=cfg.clip_grad_norm, grad_flat=reducer.flat)
    seqs, labels = [], []
    for v in range(args.videos):
        f, l_ = make_video(args.T, D_IN, NCLS, cfg, seed=1 + rank * args.videos + v)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))

    def step():
        reducer.zero_grad()
        loss, _ = net(seqs, labels, compute_loss=True)
        loss.backward()
        reducer.all_reduce_mean()
        opt.step()                      # clip_grad_norm_ + Adam
        return loss

    for _ in range(args.warmup):
        step()
    S = [blk.tdu.num_seg for blk in net.block_list if hasattr(blk, "tdu")]
    log(f"[rank {rank}] TDU segments per U block: {S}")

    max_ev = args.steps * args.videos * 4 * 10 * 2 + 64
    native.check(lib.fx_prof_enable(0, max_ev), "fx_prof_enable")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms = native.D()
    fl = native.D()
    by = native.D()
    cnt = native.I()
    import ctypes
    native.check(lib.fx_prof_collect(0, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by), ctypes.byref(cnt)),
                 "fx_prof_collect")
    lib.fx_prof_disable()
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    frames = world * args.videos * args.T * args.steps
    value = frames / elapsed
    if rank == 0:
        avg_ms = ms.value / max(cnt.value, 1)
        flops_per_launch = fl.value / max(cnt.value, 1)
        achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
        roofline = dict(bound="mfma", achieved=round(achieved, 2), peak=F32_MFMA_PEAK_TFLOPS, unit="TFLOP/s",
                        frac=round(achieved / F32_MFMA_PEAK_TFLOPS, 4),
                        traffic=(traffic_from_profiles(DOMINANT_KERNEL) if args.T == T_DEFAULT and args.videos == 2 else None),
                        kernel=DOMINANT_KERNEL + " (implicit dilated-conv GEMM: MS-TCN conv fwd + conv dX)",
                        launches=cnt.value, avg_launch_ms=round(avg_ms, 5),
                        flops_per_launch=flops_per_launch)
        line = dict(metric=METRIC, value=round(value, 1), unit="frames/s", n_gpus=world, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(1e3 * elapsed / args.steps, 3), higher_is_better=True,
                    scaling="weak", vs_baseline=None, dtype="fp32", data="synthetic",
                    config=dict(workload=f"FACT_CLIP HAViD-holdout dims, seg10 synthetic, T={args.T}",
                                model="FACT_CLIP", T=args.T, D=D_IN, Nact=NTOKEN, C=NCLS,
                                videos_per_rank=args.videos, global_batch=world * args.videos, seq_len=args.T,
                                parallelism=f"dp{world}", tdu_segments=S),
                    roofline=roofline)
        if world == 1 and not args.no_cpu_baseline:
            cb, step_flops = cpu_baseline(args.T)
            line["cpu_baseline"] = cb
            step_time = elapsed / args.steps
            line["step_mfma_frac"] = round(step_flops * args.videos / step_time / 1e12 / F32_MFMA_PEAK_TFLOPS, 5)
            line["step_gflop_per_video"] = round(step_flops / 1e9, 2)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
