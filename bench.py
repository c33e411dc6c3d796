#!/usr/bin/env python
"""Benchmark: FACT_CLIP forward + loss + backward (+ gradient all-reduce) frames/s on MI355X.

Workload (BASELINE.json metric, SURVEY.md section 8d "primary"): FACT_CLIP with
the HAViD view0_lh_pt_holdout dims and FACT.ntoken 32 (H=512, A=F=256, FF=512,
8 heads, 10 TCN layers, blocks iuUU), D=2048, C=75, T=4096 frames per video,
synthetic "seg10" videos (10 ground-truth segments, piecewise-constant
features), random-init weights (torch.manual_seed), fp32 parity arithmetic,
dropout / channel masking / time mask off (as in the reference CPU baseline).

One timed step = zero_grad + forward + loss + backward over
``--videos`` videos per rank (+ the gradient all-reduce for N>1), with the weights
FIXED, so the data-dependent TDU segment counts S stay those of the initial weights
(bench asserts they equal the CPU oracle's).  The reference train step's
clip_grad_norm_(10) + Adam(lr 1e-4) (scripts/train.py:265-268) is timed separately
afterwards and reported as the extra key ``train_step_with_adam`` (its updates move
the weights and therefore S; the S it ends with is reported there).

  python bench.py [--gpus N --steps K --warmup W]
  python bench.py --config breakfast         # BASELINE configs[0]: vanilla FACT, T=512
  python bench.py --config shipped           # havid_view0_lh_pt_holdout.yaml as shipped (training mode)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

``python bench.py --gpus N`` (N > 1, no launcher environment) starts the N ranks itself as a
torchrun child before anything touches the GPU, and refuses (exit 2) when fewer than N GPUs are
visible or when WORLD_SIZE disagrees with --gpus.  Rank 0 prints one JSON line.  ``value`` = all frames processed by all ranks /
max-over-ranks wall time of the K timed steps.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

# PMC summaries under profiles/ (tools/pmc_dominant.sh): the fused MS-TCN layer kernel (the dominant
# kernel since round 4) in pmc_dominant.json, the dilated-conv GEMM in pmc_conv_gemm.json
CONV_KERNEL = "gemm_f32_wide8_kernel<1, 0, 0>"   # rocprofv3 name: fx::(anonymous namespace)::gemm_f32_wide8_kernel<1, 0, 0>
FRL_KERNEL = "frl_kernel"
METRIC = "frames/sec FACT_CLIP fwd+bwd, T=4096 D=2048 Nact=32, at 1/2/4/8 GPUs"
METRIC_BREAKFAST = "frames/sec FACT fwd+bwd, Breakfast dims T=512 D=2048 Nact=60 (BASELINE configs[0])"
METRIC_SHIPPED = ("frames/sec FACT_CLIP fwd+bwd, havid_view0_lh_pt_holdout.yaml as shipped (ntoken 75, dropout 0.2, "
                  "cmr 0.3, time mask on), ragged T=4096+2900 D=2048")
SHIPPED_RATIO = 2900 / 4096      # second video's length relative to --T (a ragged batch, dataset.py:106-131)
F32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
BF16_MFMA_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: dense bf16 MFMA peak (no sparsity)
SPLIT_PRODUCTS = 6               # FX_PREC_F32S: bf16 piece products per fp32 product
SPLIT_KERNEL = "gemm_split_wide8_kernel<1, 0, 3>"
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: HBM3E 8 TB/s spec
HOLDOUT = [51, 53, 61, 67, 56]   # havid_view0_lh_pt_holdout.yaml
# fx_prof kinds of the X2Y attention cores (capi.cpp fx_x2y_fwd / fx_x2y_bwd); algorithmic bytes per call:
# query, key and value rows, the logit / probability tiles and the attended features (+ their gradients)
# frame-level calls (max(Nx, Ny) >= 1024: the Update block's 2 x 4096-frame maps) and segment-level calls (the TDU
# blocks' maps over the segments) are separate kinds, so each line's bytes and time come from one call shape
X2Y_KINDS = {3: "x2y_a2f_fwd", 4: "x2y_a2f_bwd", 5: "x2y_f2a_fwd", 6: "x2y_f2a_bwd",
             11: "x2y_a2f_fwd_seg", 12: "x2y_a2f_bwd_seg", 13: "x2y_f2a_fwd_seg", 14: "x2y_f2a_bwd_seg"}
FRL_KIND = 7   # fx_prof kind of the fused MS-TCN layer kernel (mstcn_fused.hip)
# fx_prof kinds of the cross-attention projection GEMMs (north-star measurement set)
XATTN_KINDS = {9: "sca_kv_projection", 10: "x2y_projections"}
XATTN_NOTES = {
    "sca_kv_projection": ("SCA frame-memory K/V projection: every decoder layer's keys and values in one frame-level "
                          "GEMM (basic.py:508-516 in-projection of the memory), gemm_f32 wide kernel",
                          "r05_pmc_kvproj.json"),
    "x2y_projections": ("X2Y_map input projections k, v (X rows) and q (Y rows) (basic.py:357-369), three GEMMs "
                        "per call", "r05_pmc_x2yproj.json"),
}
X2Y_NOTES = {"x2y_a2f_fwd": "x2y_a2f_kernel<0> (frames attend to the action tokens: logit, attn, feat in one launch)",
             "x2y_a2f_bwd": "x2y_a2f_kernel<1> + x2y_a2f_dw_kernel (weight-side dxv / dxk in one launch)",
             "x2y_f2a_fwd": "x2y_f2a_chunk_kernel + x2y_f2a_merge_kernel (tokens attend to the frames)",
             "x2y_f2a_bwd": "x2y_f2a_bwd_kernel (one launch: dP in LDS across a grid barrier, softmax backward, "
                            "dxv / dxk / dyq partials) + x2y_f2a_bwd_merge_kernel"}
for _k in list(X2Y_NOTES):
    X2Y_NOTES[_k + "_seg"] = X2Y_NOTES[_k] + " -- segment-level calls (TDU blocks)"
D_IN, NCLS, NTOKEN, T_DEFAULT = 2048, 75, 32, 4096
BF_NCLS, BF_NTOKEN, BF_T = 48, 60, 512   # breakfast.yaml (FACT.ntoken 60, 48 classes)


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


def make_cfg_breakfast():
    """fact_clip/configs/breakfast.yaml (vanilla FACT: MS-TCN++ frame branch 'm2', hid/a/f dim 512,
    ntoken 60, 48 classes) with cmr / time mask off, as the CPU reference baseline runs."""
    from factmx.configs import get_cfg_defaults
    cfg = get_cfg_defaults()
    cfg.Bi.update(dict(hid_dim=512, dropout=0.0, a="sca", a_nhead=8, a_ffdim=512, a_layers=6, a_dim=512,
                       f="m2", f_layers=10, f_ln=False, f_dim=512, f_ngp=1))
    for blk in (cfg.Bu, cfg.BU):
        blk.update(dict(a="sa", a_dim=None, a_ffdim=None, a_layers=1, a_nhead=8, dropout=None, f=None,
                        f_dim=None, f_layers=10, f_ln=None, f_ngp=None, hid_dim=None))
    cfg.BU.s_layers = 1
    cfg.FACT.update(dict(block="iuUU", cmr=0.0, fpos=False, mwt=0.1, ntoken=BF_NTOKEN, trans=False))
    cfg.Loss.update(dict(a2fc=1.0, bgw=1.0, match="o2o", pc=0.2, sw=5.0))
    cfg.Loss.nullw = BF_NTOKEN / ((BF_NTOKEN - 10) * BF_NCLS)
    cfg.TM.use = False
    cfg.holdout_mode = False
    cfg.holdout_classes = []
    cfg.use_clip = False
    cfg.batch_size = 4
    cfg.lr = 1e-4
    cfg.optimizer = "Adam"
    cfg.clip_grad_norm = 10.0
    return cfg


def make_video(T, D, C, cfg, seed, nseg=10, data="seg10"):
    """seg10 synthetic video: 10 segments with sorted random cut points,
    one randn(D) prototype per segment, labels seen[(7i+3) % |seen|].  data="iid": the stress input of
    the same section -- features ~ N(0, 1) i.i.d. (a fresh generator on the same seed), the same labels
    (thousands of TDU segments per block: the BiGRU over segments dominates)."""
    g = torch.Generator().manual_seed(seed)
    hold = set(getattr(cfg, "holdout_classes", []) or [])
    seen = [c for c in range(C) if c not in hold]
    cuts = torch.sort(torch.randperm(T - 1, generator=g)[: nseg - 1] + 1).values.tolist()
    bounds = [0] + cuts + [T]
    protos = torch.randn(nseg, D, generator=g)
    feats = torch.empty(T, D)
    label = torch.empty(T, dtype=torch.int64)
    for i in range(nseg):
        feats[bounds[i]:bounds[i + 1]] = protos[i]
        label[bounds[i]:bounds[i + 1]] = seen[(7 * i + 3) % len(seen)]
    if data == "iid":
        feats = torch.randn(T, D, generator=torch.Generator().manual_seed(seed))
    return feats.numpy(), label.numpy()


def text_embeddings(C):
    g = torch.Generator().manual_seed(0)
    t = torch.randn(C, 512, generator=g)
    return t / t.norm(dim=1, keepdim=True)


def build_model(cfg, D, C, device, seed=0, clip=True):
    from factmx.models.blocks import FACT, FACT_CLIP
    from factmx.models.loss import MatchCriterion
    text = text_embeddings(C)
    torch.manual_seed(seed)
    net = FACT_CLIP(cfg, D, C, text_embeddings=text.clone()) if clip else FACT(cfg, D, C)
    net.mcriterion = MatchCriterion(cfg, C, [])
    return net.to(device), text


def make_cfg_shipped():
    """havid_view0_lh_pt_holdout.yaml exactly as the reference ships it for training: ntoken 75,
    Bi.dropout 0.2, FACT.cmr 0.3 (Dropout2d channel masking), time mask on (m 5, p 0.05, t 30),
    Loss.nullw -1 (derived by train_tools.py:54-71 from the transcript length, here 10)."""
    cfg = make_cfg(ntoken=75)
    cfg.Bi.dropout = 0.2
    cfg.FACT.cmr = 0.3
    cfg.TM.update(dict(use=True, inplace=True, m=5, p=0.05, t=30))
    return cfg


def workload(name):
    """(cfg, D, C, T default, videos per rank, FACT_CLIP?, metric) of a named bench workload."""
    if name == "breakfast":
        return make_cfg_breakfast(), D_IN, BF_NCLS, BF_T, 4, False, METRIC_BREAKFAST
    if name == "shipped":
        return make_cfg_shipped(), D_IN, NCLS, T_DEFAULT, 2, True, METRIC_SHIPPED
    return make_cfg(), D_IN, NCLS, T_DEFAULT, 2, True, METRIC


def video_lengths(name, T, nv):
    """Frames of each video of a rank's step: equal lengths, except the shipped config's ragged pair."""
    if name == "shipped":
        return [T if v % 2 == 0 else int(round(T * SHIPPED_RATIO)) for v in range(nv)]
    return [T] * nv


def video_segments(net):
    """Per-video TDU segment counts of the last forward: [[S of each U block] for each video]."""
    return [list(s) for s in getattr(net, "video_segments", [])]


def traffic_from_profiles(kernel_prefix, name="pmc_dominant.json"):
    """HBM bytes per launch of a kernel from a committed rocprofv3 PMC summary (FETCH_SIZE / WRITE_SIZE
    passes, tools/pmc_dominant.sh), if any."""
    path = os.path.join(ROOT, "profiles", name)
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


PREC_NOTES = {
    "bf16": ("bf16 products, fp32 accumulation/storage (FX_PREC_BF16)",
             "same weights and videos as the headline line; weight-gradient GEMMs, attention, normalisation and "
             "losses stay fp32"),
    "fp32": ("fp32 (every GEMM product on the f32 MFMA, FX_PREC_F32)",
             "same weights and videos as the headline line, frame-level GEMMs on v_mfma_f32_32x32x2_f32"),
    "fp32s": ("fp32 (frame-level GEMMs on the bf16 matrix cores by a 3-piece split, FX_PREC_F32S)",
              "same weights and videos as the headline line"),
}


def bf16_mode(net, step, frames_per_step, steps, warmup, fxf, mode="bf16"):
    """Time `steps` fixed-weight steps with the current stream's GEMM precision set to `mode` and compare
    its frame logits (last block, every video) and TDU segment counts with the headline precision's."""
    # the same random draws for both runs (dropout seeds come from torch's CPU generator, Dropout2d from
    # the CUDA one, the time mask from Python's `random`, basic.py time_mask): under a stochastic config
    # both precisions then see identical masks
    import random
    rng = (torch.get_rng_state(), torch.cuda.get_rng_state(), random.getstate())

    def logits():
        torch.set_rng_state(rng[0])
        torch.cuda.set_rng_state(rng[1])
        random.setstate(rng[2])
        step()
        torch.cuda.synchronize()
        last = net.block_list[-1]
        recs = getattr(last, "_vrec", None)   # lockstep batch: every video; else the last video run
        z = [r["frame_clogit"] for r in recs] if recs else [last.frame_clogit]
        return [t.detach().clone() for t in z], video_segments(net)
    z32, s32 = logits()
    with fxf.gemm_precision(mode):
        z16, s16 = logits()
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    dev = max((a - b).abs().max().item() for a, b in zip(z16, z32))
    scale = max(b.abs().max().item() for b in z32)
    agree = sum(int((a.argmax(-1) == b.argmax(-1)).sum()) for a, b in zip(z16, z32)) / sum(b.shape[0] for b in z32)
    dtype, note = PREC_NOTES[mode]
    return dict(value=round(frames_per_step * steps / el, 1), unit="frames/s", ms_per_step=round(1e3 * el / steps, 3),
                dtype=dtype, frame_logit_max_abs_dev=round(dev, 6), frame_logit_max_abs=round(scale, 4),
                frame_argmax_agreement=round(agree, 5), tdu_segments=s16, tdu_segments_headline=s32, note=note)


def dp_schedule_overhead(net, seqs, labels, steps, rounds=3):
    """N=1 only: the data-parallel schedule run for real over RCCL in a one-rank ``nccl`` group --
    per-block bucket all-reduces (AVG) launched from the backward hooks on a collective stream that
    waits for the compute and side streams -- against the plain step (schedule off), in alternating
    rounds of `steps` steps.  Returns the overhead (median forced - median plain, ms/step)."""
    import statistics
    import torch.distributed as dist
    from factmx.dp import DataParallel
    dev = seqs[0].device
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        dp = DataParallel(net, broadcast=False, force_buckets=True)

        def step():
            dp.zero_grad()
            loss, _ = net(seqs, labels, compute_loss=True)
            loss.backward()
            dp.finish_gradients()

        def timed(active):
            dp.active = active
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            return 1e3 * (time.perf_counter() - t0) / steps
        plain, forced = [], []
        for _ in range(rounds):
            plain.append(timed(False))
            forced.append(timed(True))
        early = [k if isinstance(k, int) else f"{k[0]}.{k[1]}" for k in dp.hook_launched]
        pm, fm = statistics.median(plain), statistics.median(forced)
        return dict(dp_schedule_overhead_ms=round(fm - pm, 3), plain_ms_per_step=[round(v, 3) for v in plain],
                    forced_ms_per_step=[round(v, 3) for v in forced], backend=dist.get_backend(),
                    buckets_per_step=sum(len(b) for b in dp.block_buckets.values()) + len(dp.rest_buckets),
                    hook_launched_blocks=early,
                    dp_tail_mb=round(dp.tail_bytes / 2 ** 20, 2),
                    dp_total_mb=round(dp.flat.numel() * dp.flat.element_size() / 2 ** 20, 2),
                    note="world-size-1 nccl (RCCL) group, DataParallel(force_buckets=True): every block's bucket "
                         "all-reduced (AVG) from its backward hook; median of alternating rounds")
    finally:
        dist.destroy_process_group()


# The kernels of each timed call kind, as the rocprofv3 kernel trace names them: `frac` of the attention-over-T
# and frame-level X2Y lines is taken from the committed trace of this bench shape (profiles/r06_trace_kernels.json,
# tools/r06_diag.sh: per kernel the largest grid = the frame-level call), the live event timing is reported beside it
TRACE_KERNELS = {"fwd": ["tattn_fwd32_kernel<2>"], "bwd": ["tattn_bwd32_kernel<2>"],
                 "x2y_a2f_fwd": ["x2y_a2f_kernel<0>"], "x2y_a2f_bwd": ["x2y_a2f_kernel<1>", "x2y_a2f_dw_kernel"],
                 "x2y_f2a_fwd": ["x2y_f2a_chunk_kernel", "x2y_f2a_merge_kernel"],
                 "x2y_f2a_bwd": ["x2y_f2a_bwd_kernel<3>", "x2y_f2a_bwd_merge_kernel"],
                 "frl": ["frl_kernel<true, 3>"]}
TRACE_FILE = "r06_trace_kernels.json"


def trace_call_us(name):
    """Kernel time of one call of kind `name` from the committed kernel trace (sum over its kernels of each
    kernel's average duration at its largest grid), or None."""
    path = os.path.join(ROOT, "profiles", TRACE_FILE)
    if name not in TRACE_KERNELS or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            ks = json.load(f)["kernels"]
        tot = 0.0
        for k in TRACE_KERNELS[name]:
            grids = ks[k]
            tot += grids[max(grids, key=int)][1]
        return tot
    except (OSError, ValueError, KeyError):
        return None


def trace_basis(entry, name, per_call, peak, unit_scale):
    """Re-base a roofline entry's `frac` on the committed kernel trace (per_call: algorithmic bytes or FLOPs of
    one call; unit_scale 1e9 for GB/s, 1e12 for TFLOP/s); the live event-based values stay as `live_*`."""
    us = trace_call_us(name)
    if entry is None or us is None:
        return entry
    ach = per_call / (us * 1e-6) / unit_scale
    entry.update(live_achieved=entry["achieved"], live_frac=entry["frac"], live_avg_launch_ms=entry["avg_launch_ms"],
                 achieved=round(ach, 2), frac=round(ach / peak, 4), avg_launch_ms=round(us / 1e3, 5),
                 basis=f"rocprofv3 kernel-trace average of this shape's kernels (profiles/{TRACE_FILE}); live_*: "
                       "hipExtLaunchKernel event pairs in the first timed step (they read ~2-5 us per kernel over the "
                       "trace on this part)")
    return entry


class Prof:
    """One fx_prof kind over the sampled step(s): the calls' event brackets (kernels + any host-issue gap
    inside the call) and the kernels alone (each kernel's own hipExtLaunchKernel event pair: its execution
    time, as the rocprofv3 kernel trace reports it).  Every roofline below is on the KERNEL basis."""

    def __init__(self, bracket_ms=0.0, flops=0.0, nbytes=0.0, calls=0, kernel_ms=0.0, kernels=0, untimed=0):
        self.bracket_ms, self.flops, self.bytes, self.calls = bracket_ms, flops, nbytes, calls
        self.kernel_ms, self.kernels, self.untimed = kernel_ms, kernels, untimed

    def timing(self):
        """Fields every roofline entry carries: per call, kernel time and the host gap inside the bracket."""
        n = max(self.calls, 1)
        return dict(basis="kernel time (hipExtLaunchKernel event pairs, = rocprofv3 kernel-trace durations)",
                    kernel_ms_per_call=round(self.kernel_ms / n, 5), bracket_ms_per_call=round(self.bracket_ms / n, 5),
                    host_gap_ms_per_call=round(max(self.bracket_ms - self.kernel_ms, 0.0) / n, 5),
                    kernels_per_call=round(self.kernels / n, 2), untimed_kernels=self.untimed)


def prof_collect(lib, kind):
    """The Prof of one profiling kind (HIP-event brackets of its calls + the kernel-time pairs inside)."""
    from factmx import native
    ms, fl, by, cnt = native.D(), native.D(), native.D(), native.I()
    native.check(lib.fx_prof_collect(kind, ctypes.byref(ms), ctypes.byref(fl), ctypes.byref(by),
                                     ctypes.byref(cnt)), "fx_prof_collect")
    kms, kn, ku = native.D(), native.I(), native.I()
    native.check(lib.fx_prof_collect_kernels(kind, ctypes.byref(kms), ctypes.byref(kn), ctypes.byref(ku)),
                 "fx_prof_collect_kernels")
    return Prof(ms.value, fl.value, by.value, cnt.value, kms.value, kn.value, ku.value)


def attention_roofline(kernel, pr):
    """Attention over T (SCA cross-attention) and the X2Y cores: HBM-bound, algorithmic
    bytes per call over the KERNEL time of the call (its kernels' summed durations)."""
    n = max(pr.calls, 1)
    avg_ms = pr.kernel_ms / n
    if pr.calls <= 0 or avg_ms <= 0:
        return None
    gbs = pr.bytes / n / (avg_ms * 1e-3) / 1e9
    return dict(kernel=kernel, bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(gbs / HBM_PEAK_GBS, 4),
                traffic=None, launches=pr.calls, avg_launch_ms=round(avg_ms, 5), bytes_per_launch=pr.bytes / n,
                tflops=round(pr.flops / n / (avg_ms * 1e-3) / 1e12, 2), **pr.timing())


def fused_layer_roofline(pr, peak):
    """The fused MS-TCN layer kernel (mstcn_fused.hip: conv + ReLU + 1x1 + residual in one launch, and
    the fused dX chain of the backward), MFMA-bound: 2 rows F 4F algorithmic FLOPs per launch (the
    3-tap conv's 3F and the 1x1's F columns) over its kernel time; None when the two-GEMM layers ran."""
    n = pr.calls
    if n <= 0 or pr.bracket_ms <= 0:
        return None
    # live: one event pair around each back-to-back chain of a stack's fused-layer launches (the host issues the
    # whole chain from one C call, so the bracket is kernel time plus the launches' dispatch gaps)
    avg_ms = pr.bracket_ms / n
    tf = pr.flops / n / (avg_ms * 1e-3) / 1e12
    out = dict(kernel="frl_kernel (fused MS-TCN layer: conv fwd + 1x1 fwd, or dX chain bwd)", bound="mfma",
               achieved=round(tf, 2), peak=round(peak, 1), unit="TFLOP/s", frac=round(tf / peak, 4),
               launches=n, avg_launch_ms=round(avg_ms, 5), flops_per_launch=pr.flops / n,
               bytes_per_launch=pr.bytes / n, basis="HIP events around the back-to-back fused-layer chains")
    us = trace_call_us("frl")
    if us is not None:        # cross-check: the committed kernel trace of this shape
        out.update(trace_avg_launch_ms=round(us / 1e3, 5),
                   trace_frac=round(pr.flops / n / (us * 1e-6) / 1e12 / peak, 4))
    return out


def gemm_roofline(name, pr, peak):
    """A cross-attention projection GEMM kind, MFMA-bound: algorithmic FLOPs over the HIP-event time of its
    launches in the sampled step(s); `traffic` from a committed standalone PMC pass of the same shape."""
    n = pr.calls
    if n <= 0 or pr.bracket_ms <= 0:
        return None
    note, pmc = XATTN_NOTES[name]
    ms = pr.bracket_ms
    tf = pr.flops / (ms * 1e-3) / 1e12
    out = dict(kernel=note, bound="mfma", achieved=round(tf, 2), peak=round(peak, 1), unit="TFLOP/s",
               frac=round(tf / peak, 4), launches=n, avg_launch_ms=round(ms / n, 5),
               flops_per_launch=pr.flops / n, bytes_per_launch=pr.bytes / n,
               hbm_gbs_algorithmic=round(pr.bytes / (ms * 1e-3) / 1e9, 1))
    path = os.path.join(ROOT, "profiles", pmc)
    out["traffic"] = None
    if os.path.exists(path):
        try:
            with open(path) as f:
                out["traffic"] = json.load(f).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
    return out


def cpu_baseline(wl, Ts, videos_seeds, min_seconds=10.0, min_steps=2, data="seg10"):
    """The CPU oracle (fp32 PyTorch restatement pinned to the reference) timed on host cores: one
    video per step, full T, forward + prediction + loss + backward with FIXED weights (the same
    unit as the GPU step), repeated until >= min_seconds of CPU work (a bounded sample).  Also
    returns the algorithmic FLOPs of one video step and the oracle's TDU segment counts of every
    bench video at the initial weights."""
    from torch.utils.flop_counter import FlopCounterMode
    from oracle import fact_oracle as fo
    cfg, D, C, _, _, clip, _ = workload(wl)
    net, text = build_model(cfg, D, C, "cpu", seed=0, clip=clip)
    spec = fo.resolve_spec(cfg, D, C, clip=clip)
    P = {n: p.detach().clone().float().requires_grad_(True) for n, p in net.named_parameters()}
    txt = text if clip else None
    vids = [make_video(Tv, D, C, cfg, seed=s, data=data) for Tv, s in zip(Ts, videos_seeds)]

    def step(v=0):
        for p in P.values():
            p.grad = None
        out = fo.forward(spec, P, torch.from_numpy(vids[v][0]))
        fo.predict(spec, out, txt)
        total, _, _, _ = fo.video_loss(spec, out, vids[v][1], txt)
        total.backward()
        return out

    S = []
    with torch.no_grad():
        for f, _ in vids:
            out = fo.forward(spec, P, torch.from_numpy(f))
            S.append([len(r["tdu"].starts) for r in out["blocks"] if r["type"] == "U"])
    flops = 0          # algorithmic FLOPs of one step over every bench video
    for v in range(len(vids)):
        with FlopCounterMode(display=False) as fc:
            step(v)
        flops += fc.get_total_flops()
    t0 = time.perf_counter()
    n = frames = 0
    while n < min_steps or time.perf_counter() - t0 < min_seconds:
        step(n % len(vids))
        frames += Ts[n % len(vids)]
        n += 1
    dt = time.perf_counter() - t0
    stoch = " (the oracle has no dropout / channel masking / time mask: those stay off in the CPU sample)" \
        if wl == "shipped" else ""
    return dict(value=round(frames / dt, 1), unit="frames/s", cores=torch.get_num_threads(), kind="port",
                sample=f"{n} steps x 1 video (T={'/'.join(str(t) for t in sorted(set(Ts)))}, {data}, the bench videos "
                       f"in turn) fwd+loss+bwd, fixed weights, oracle fp32 (1 untimed warm-up step, {dt:.1f} s "
                       f"timed){stoch}"), flops, S


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """``--gpus N`` without a torch.distributed launcher: start N ranks (one process per GPU) as a
    torchrun child and return its exit code.  Runs BEFORE anything touches the GPU (counting devices
    does not initialise it); refuses loudly when fewer than N GPUs are visible, so an N-GPU request is
    never timed as one rank."""
    import subprocess
    visible = torch.cuda.device_count()
    if visible < n:
        log(f"bench.py: --gpus {n} requested but only {visible} GPU(s) are visible; refusing to time "
            f"fewer ranks than requested")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    log("bench.py: launching " + " ".join(cmd))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=["havid", "breakfast", "shipped"], default="havid",
                    help="havid: FACT_CLIP T=4096 (the BASELINE metric); breakfast: vanilla FACT T=512; "
                         "shipped: the reference's havid holdout yaml unchanged (dropout, cmr, time mask, "
                         "ntoken 75), ragged T=4096+2900")
    ap.add_argument("--videos", type=int, default=None, help="videos per rank per step (yaml batch_size)")
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--data", choices=["seg10", "iid"], default="seg10",
                    help="seg10: the headline's synthetic videos; iid: the stress input (features i.i.d. N(0, 1), "
                         "thousands of TDU segments, BiGRU-bound)")
    ap.add_argument("--adam-steps", type=int, default=None,
                    help="extra timed steps with clip_grad_norm_ + Adam after the fixed-weight steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-bf16", action="store_true", help="skip the extra precision-mode measurements (N=1 only)")
    ap.add_argument("--no-dp-overhead", action="store_true",
                    help="skip the N=1 RCCL measurement of the data-parallel bucket schedule")
    ap.add_argument("--prec", choices=["default", "fp32s", "fp32"], default="default",
                    help="GEMM arithmetic of the headline: the library default, fp32s (fp32 by a 3-piece bf16 split "
                         "on the bf16 matrix cores) or fp32 (f32 MFMA)")
    args = ap.parse_args()
    cfg, D, C, T_def, vids_def, clip, metric = workload(args.config)
    T = args.T or T_def
    nv = args.videos or vids_def
    adam_steps = args.steps if args.adam_steps is None else args.adam_steps

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per requested GPU")
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    from factmx import native
    from factmx import functional as fxf_
    from factmx.dp import DataParallel
    from factmx.optim import FusedAdam
    lib = native.load()
    if args.prec != "default":
        fxf_.set_default_precision(args.prec)
    headline_prec = fxf_.default_precision()

    net, _ = build_model(cfg, D, C, dev, seed=0, clip=clip)
    net.train()
    dp = DataParallel(net)      # flat gradient buckets (+ rank-0 weight broadcast, overlapped all-reduce)
    seeds = [1 + rank * nv + v for v in range(nv)]
    Ts = video_lengths(args.config, T, nv)
    seqs, labels = [], []
    for s, Tv in zip(seeds, Ts):
        f, l_ = make_video(Tv, D, C, cfg, seed=s, data=args.data)
        seqs.append(torch.from_numpy(f).to(dev))
        labels.append(torch.from_numpy(l_).to(dev))

    def step():
        dp.zero_grad()
        loss, _ = net(seqs, labels, compute_loss=True)
        loss.backward()
        dp.finish_gradients()           # bucket all-reduces (mean) for N>1
        return loss

    for _ in range(args.warmup):
        step()
    # the host heap built so far (torch, the model, the warm-up's caches) is long-lived: move it out of
    # the cyclic collector's generations so a full collection does not stall a step for ~60 ms walking
    # it (factmx.utils.runtime.freeze_host_heap; round-4 diagnosis of the Adam leg)
    from factmx.utils.runtime import freeze_host_heap
    freeze_host_heap()
    S = video_segments(net)
    log(f"[rank {rank}] TDU segments per video (per U block): {S}")

    # HIP events around the dominant kernel's launches (and the attention / X2Y launches) of the FIRST timed
    # step(s) only: an event pair per launch costs host time (~1 ms per step over all 80 conv launches,
    # A/B in DESIGN.md), so the roofline samples the timed region instead of perturbing all of it
    # (FX_BENCH_PROF_STEPS: steps to sample; the durations agree with the all-steps sampling).  The event
    # capacity of each kind is its launch count in one step, counted on an untimed extra warm-up step,
    # times the sampled steps -- so no event pair spills into the later timed steps.
    psteps = min(args.steps, int(os.environ.get("FX_BENCH_PROF_STEPS", 1)))
    kinds = [0, 1, 2] + list(X2Y_KINDS) + [FRL_KIND] + list(XATTN_KINDS)
    for kind in kinds:
        native.check(lib.fx_prof_enable(kind, 4096), "fx_prof_enable")
    step()
    per_step = {kind: prof_collect(lib, kind).calls for kind in kinds}
    lib.fx_prof_disable()
    for kind in kinds:
        if per_step[kind] > 0:
            native.check(lib.fx_prof_enable(kind, per_step[kind] * psteps), "fx_prof_enable")
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
    def collect(kind):
        if per_step[kind] > 0:
            return prof_collect(lib, kind)
        return Prof()
    conv_prof = collect(0)
    attn_prof = {name: collect(kind) for kind, name in ((1, "fwd"), (2, "bwd"))}
    x2y_prof = {name: collect(kind) for kind, name in X2Y_KINDS.items()}
    frl_prof = collect(FRL_KIND)
    xattn_prof = {name: collect(kind) for kind, name in XATTN_KINDS.items()}
    lib.fx_prof_disable()
    S_after = video_segments(net)
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()

    # the reference train step (clip_grad_norm_ + Adam), timed right after the fixed-weight steps (same
    # device state); the weights are restored afterwards, so the precision modes below compare
    # arithmetic on the headline's weights
    adam = None
    if adam_steps > 0:
        w0 = [p.detach().clone() for p in net.parameters()]
        opt = FusedAdam(net.parameters(), lr=cfg.lr, max_grad_norm=cfg.clip_grad_norm, grad_flat=dp.flat)
        step()
        opt.step()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ta = time.perf_counter()
        for _ in range(adam_steps):
            step()
            opt.step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        ea = time.perf_counter() - ta
        if world > 1:
            t = torch.tensor([ea], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ea = t.item()
        adam = dict(value=round(world * sum(Ts) * adam_steps / ea, 1), unit="frames/s", steps=adam_steps,
                    ms_per_step=round(1e3 * ea / adam_steps, 3), tdu_segments_after=video_segments(net),
                    note="zero_grad + fwd + loss + bwd (+all-reduce) + clip_grad_norm_(10) + Adam(lr 1e-4); the "
                         "updates move the weights, so S drifts from the fixed-weight value")
        with torch.no_grad():
            for p_, w in zip(net.parameters(), w0):
                p_.copy_(w)
        del opt, w0

    # BASELINE configs[1]: the same fixed-weight step with the frame-level GEMMs in bf16 arithmetic
    # (FX_PREC_BF16, fp32 accumulation / storage), its frame-logit deviation from the fp32 path on the
    # same weights and videos, and its TDU segment counts (N=1 only; the headline stays fp32)
    bf16 = other = None
    if world == 1 and not args.no_bf16:
        from factmx import functional as fxf
        bf16 = bf16_mode(net, step, sum(Ts), args.steps, args.warmup, fxf)
        # the other fp32 arithmetic (f32 MFMA when the headline runs the split, and vice versa)
        other = bf16_mode(net, step, sum(Ts), args.steps, args.warmup, fxf,
                          "fp32" if headline_prec == "fp32s" else "fp32s")

    dp_sched = None
    if world == 1 and not args.no_dp_overhead:
        try:
            dp_sched = dp_schedule_overhead(net, seqs, labels, args.steps)
        except Exception as e:          # reported, never fatal for the headline line
            dp_sched = dict(error=f"{type(e).__name__}: {e}")

    frames = world * sum(Ts) * args.steps
    value = frames / elapsed
    if rank == 0:
        avg_ms = conv_prof.bracket_ms / max(conv_prof.calls, 1)
        flops_per_launch = conv_prof.flops / max(conv_prof.calls, 1)
        achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
        default_shape = args.config == "havid" and T == T_DEFAULT and nv == 2 and args.data == "seg10"
        split = headline_prec == "fp32s"
        # split arithmetic: the matrix cores' bound is the bf16 dense peak over the 6 piece products
        # (fp32 FLOPs counted once); f32 MFMA: the f32 matrix peak
        peak = BF16_MFMA_PEAK_TFLOPS / SPLIT_PRODUCTS if split else F32_MFMA_PEAK_TFLOPS
        conv_roofline = dict(bound="mfma", achieved=round(achieved, 2), peak=round(peak, 1), unit="TFLOP/s",
                        frac=round(achieved / peak, 4),
                        traffic=(traffic_from_profiles(SPLIT_KERNEL if split else CONV_KERNEL,
                                                       "pmc_split.json" if split else "pmc_conv_gemm.json")
                                 if default_shape else None),
                        kernel=(f"{SPLIT_KERNEL} (implicit dilated-conv GEMM in fp32 by 3-piece bf16 split: conv fwd "
                                f"+ conv dX; peak = bf16 dense peak / {SPLIT_PRODUCTS} products)" if split else
                                "gemm_f32_wide8_kernel (implicit dilated-conv GEMM: conv fwd + conv dX of the layers "
                                "the fused MS-TCN layer kernel does not run)"),
                        launches=conv_prof.calls, avg_launch_ms=round(avg_ms, 5),
                        flops_per_launch=flops_per_launch,
                        sample=f"HIP events around the conv-GEMM launches of the first timed step ({conv_prof.calls})")
        # the dominant kernel by measured time in the sampled step: the fused MS-TCN layer when it ran
        frl_roofline = fused_layer_roofline(frl_prof, F32_MFMA_PEAK_TFLOPS)
        if frl_roofline is not None:
            frl_roofline["traffic"] = traffic_from_profiles(FRL_KERNEL) if default_shape else None
            frl_roofline["sample"] = (f"{frl_roofline['launches']} fused-layer launches from the start of the timed region "
                                      "(one event pair per MS-TCN stack and direction; the pair capacity is one "
                                      "step's launch count, so the pairs cover the first ~9 timed steps)")
        roofline = (frl_roofline if frl_roofline is not None and frl_prof.bracket_ms > conv_prof.bracket_ms
                    else conv_roofline)
        roofline_attention = {name: attention_roofline(f"tattn_{name}32_kernel (merge folded into the launch)", v)
                              for name, v in attn_prof.items()}
        for name, r in roofline_attention.items():
            if r is not None and default_shape:   # PMC bytes of the main kernel (the merge launch excluded)
                r["traffic"] = traffic_from_profiles(f"tattn_{name}32_kernel", f"r05_pmc_tattn_{name}.json")
                trace_basis(r, name, r["bytes_per_launch"], HBM_PEAK_GBS, 1e9)
        x2y_pmc = {}
        if default_shape and os.path.exists(os.path.join(ROOT, "profiles", "r05_pmc_x2y.json")):
            try:
                with open(os.path.join(ROOT, "profiles", "r05_pmc_x2y.json")) as f:
                    x2y_pmc = json.load(f)
            except (OSError, ValueError):
                x2y_pmc = {}
        for name, v in x2y_prof.items():      # the X2Y_map cores (basic.py:373-380), when they ran fused
            if v.calls > 0:
                r = roofline_attention[name] = attention_roofline(X2Y_NOTES[name], v)
                # the standalone PMC passes (tools/r05_x2y_pmc.sh) ran the frame-level call's shape (2 x 4096
                # frames, 32 tokens, head 512): comparable with the frame-level kinds only
                if r is not None and not name.endswith("_seg"):
                    r["traffic"] = x2y_pmc.get(name)
                    r["traffic_shape"] = "2 x 4096 frames x 32 tokens, Hd 512 (= this line's calls)"
                    if default_shape:
                        trace_basis(r, name, r["bytes_per_launch"], HBM_PEAK_GBS, 1e9)
        line = dict(metric=metric, value=round(value, 1), unit="frames/s", n_gpus=world, steps=args.steps,
                    warmup=args.warmup, ms_per_step=round(1e3 * elapsed / args.steps, 3), higher_is_better=True,
                    scaling="weak", vs_baseline=None, dtype="fp32", data="synthetic",
                    gemm_arithmetic=PREC_NOTES[headline_prec][0],
                    config=dict(workload=(f"FACT_CLIP havid_view0_lh_pt_holdout.yaml as shipped (training mode: "
                                          f"dropout 0.2, cmr 0.3, time mask, ntoken 75), {args.data} synthetic, "
                                          f"ragged T={'+'.join(map(str, Ts))}" if args.config == "shipped" else
                                          f"FACT_CLIP HAViD-holdout dims, {args.data} synthetic, T={T}" if clip else
                                          f"FACT (vanilla) Breakfast dims, {args.data} synthetic, T={T}"),
                                model="FACT_CLIP" if clip else "FACT", T=T, video_lengths=Ts, D=D,
                                Nact=cfg.FACT.ntoken, C=C,
                                videos_per_rank=nv, global_batch=world * nv, seq_len=T,
                                parallelism=f"dp{world}", weights="fixed (no optimizer update in the timed steps)",
                                tdu_segments=S, tdu_segments_after_timing=S_after),
                    roofline=roofline, roofline_attention=roofline_attention,
                    roofline_xattn_gemm={name: gemm_roofline(name, v, F32_MFMA_PEAK_TFLOPS)
                                         for name, v in xattn_prof.items()},
                    roofline_conv_gemm=conv_roofline, roofline_fused_layer=frl_roofline, train_step_with_adam=adam,
                    bf16_mode=bf16, dp_schedule=dp_sched)
        if other is not None:
            line["fp32_f32mfma_mode" if headline_prec == "fp32s" else "fp32_split_mode"] = other
        if world == 1 and not args.no_cpu_baseline:
            cb, step_flops, S_oracle = cpu_baseline(args.config, Ts, seeds, data=args.data)
            line["cpu_baseline"] = cb
            line["tdu_segments_oracle"] = S_oracle
            # dropout / channel masking / time mask (shipped config) draw new masks every step: S is then
            # the last timed step's, and the oracle (no stochastic layers) is no reference for it
            line["tdu_segments_match_oracle"] = None if args.config == "shipped" else S_oracle == S
            step_time = elapsed / args.steps
            line["step_mfma_frac"] = round(step_flops / step_time / 1e12 / F32_MFMA_PEAK_TFLOPS, 5)
            line["step_gflop_per_video"] = round(step_flops / nv / 1e9, 2)
            if S_oracle != S and args.config != "shipped":
                log(f"WARNING: GPU TDU segments {S} differ from the oracle's {S_oracle}")
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
