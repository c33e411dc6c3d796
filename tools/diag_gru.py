"""Diagnostic (GPU): where do the BiGRU gradients of the lockstep north-star step depart from the
fp64 oracle?  Captures the GRU input/output and their gradients on both sides (monkeypatched
wrappers, diagnostic only) for every TDU block and prints per-video max |diff| / max |ref|."""
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "fact-clip_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import numpy as np
import torch

import bench
from factmx import functional as fxf
from factmx.models import blocks as blocks_mod
from oracle import fact_oracle as fo

cap_gpu, cap_ref = [], []
orig_gpu_gru = fxf.gru
orig_ref_gru = fo.gru


def gpu_gru(mod, x, seq_off=None):
    x.retain_grad()
    y = orig_gpu_gru(mod, x, seq_off=seq_off)
    y.retain_grad()
    cap_gpu.append((x, y, seq_off))
    return y


def ref_gru(P, p, x, nl):
    x.retain_grad()
    y = orig_ref_gru(P, p, x, nl)
    y.retain_grad()
    cap_ref.append((x, y))
    return y


fxf.gru = gpu_gru
fo.gru = ref_gru
blocks_mod.fxf.gru = gpu_gru

cfg = bench.make_cfg()
T, D, C = 4096, 2048, 75
net, text = bench.build_model(cfg, D, C, device="cuda", seed=0)
net.train()
vids = [bench.make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
seqs = [torch.from_numpy(f).cuda() for f, _ in vids]
labs = [torch.from_numpy(l_).cuda() for _, l_ in vids]
loss, _ = net(seqs, labs, compute_loss=True)
loss.backward()
torch.cuda.synchronize()
from helpers import oracle_batch
spec = fo.resolve_spec(cfg, D, C, clip=True)
ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
print("loss", loss.item(), ref_loss)


def rel(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return f"maxdiff {(a - b).abs().max().item():.3e} maxref {b.abs().max().item():.3e}"


for bi, (x, y, off) in enumerate(cap_gpu):
    for v in range(2):
        rx, ry = cap_ref[v * len(cap_gpu) + bi]
        sl = slice(off[v], off[v + 1])
        print(f"TDU block {bi} video {v}: S={off[v + 1] - off[v]}")
        print("   x  ", rel(x[sl], rx))
        print("   y  ", rel(y[sl], ry), " near-zero outputs", int((ry.detach().abs() < 1e-4).sum()))
        print("   dy ", rel(y.grad[sl], ry.grad))
        print("   dx ", rel(x.grad[sl], rx.grad))
        flips = ((y[sl].detach().cpu().double() > 0) != (ry.detach() > 0)).sum().item()
        print("   relu sign flips", flips)
for n, p in net.named_parameters():
    if "seg_update" in n:
        g, r = p.grad, ref_grads[n]
        print(n, rel(g, r))
