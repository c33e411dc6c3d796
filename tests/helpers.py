"""Shared test helpers: fixture loading, config reconstruction, parameter dicts."""
import json
import os

import numpy as np
import torch

import paramgen as pg
from factmx.configs import get_cfg_defaults

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_fixture(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def tiny_meta(fx):
    return json.loads(str(fx["meta_json"]))


def cfg_from_meta(meta):
    """Rebuild the capture-time config (make_golden.make_cfg) on the product's CfgNode."""
    cfg = get_cfg_defaults()
    for sec in ("FACT", "Bi", "Bu", "BU", "Loss", "CLIP"):
        for k, v in meta.get(sec, {}).items():
            cfg[sec][k] = v
    cfg.TM.use = False
    cfg.holdout_classes = list(meta["holdout"])
    cfg.holdout_mode = bool(meta["holdout"])
    cfg.use_clip = meta["model"] == "FACT_CLIP"
    cfg.Loss.nullw = meta["nullw"]
    return cfg


def tiny_inputs(meta):
    feats, label = pg.segmented_video(meta["T"], meta["D"], meta["seen"], meta["nseg"],
                                      seed=meta["seed"], noise=meta["noise"])
    text = pg.text_embeddings(meta["C"], seed=meta["seed"])
    return feats, label, text


def param_dict(shapes, seed, dtype=torch.float64, requires_grad=True):
    P = {}
    for n, s in shapes.items():
        t = torch.from_numpy(pg.param_value(n, s, seed)).to(dtype)
        P[n] = t.requires_grad_(requires_grad)
    return P


def check_grad(fx, prefix, name, g, rtol, atol):
    """Compare a gradient with its fixture record (full, or index sample + sum/norm)."""
    g = g.detach().double().reshape(-1).numpy()
    full = f"{prefix}grad/{name}"
    if full in fx:
        np.testing.assert_allclose(g, fx[full], rtol=rtol, atol=atol, err_msg=full)
    else:
        idx = pg.sample_index(g.size)
        np.testing.assert_allclose(g[idx], fx[f"{prefix}gradsample/{name}"], rtol=rtol, atol=atol,
                                   err_msg=prefix + name)
    s, n = fx[f"{prefix}gradsum/{name}"]
    np.testing.assert_allclose(np.sqrt((g * g).sum()), n, rtol=max(rtol, 1e-6), atol=atol * np.sqrt(g.size),
                               err_msg=prefix + name + " norm")
    scale = max(abs(n), 1e-30) * np.sqrt(g.size)
    assert abs(g.sum() - s) <= max(rtol, 1e-6) * scale + atol * g.size, (prefix + name, g.sum(), s)


def oracle_batch(spec, net, vids, text=None, dtype=torch.float64):
    """The fp64 CPU oracle over a batch of videos with the GPU model's current weights, as the
    reference FACT*.forward does it (blocks.py:889-917: mean of the per-video losses): returns
    (mean loss, {param name: gradient}, [per-video forward records])."""
    from oracle import fact_oracle as fo
    P = {n: p.detach().to("cpu", dtype).requires_grad_(True) for n, p in net.named_parameters()}
    txt = None if text is None else text.to("cpu", dtype)
    outs, total = [], 0.0
    for feats, label in vids:
        out = fo.forward(spec, P, torch.from_numpy(np.asarray(feats)).to(dtype))
        t, _, _, _ = fo.video_loss(spec, out, label, txt)
        total = total + t
        outs.append(out)
    total = total / len(vids)
    total.backward()
    return float(total.detach()), {n: p.grad for n, p in P.items()}, outs


def compare_grads(net, ref, rtol=2e-3, atol_rms=1e-2, relaxed=(), relaxed_tol=2e-2, what=""):
    """Every parameter gradient of ``net`` against a reference gradient dict: a fixed sample of
    2048 entries within rtol plus an absolute floor of ``atol_rms`` x the gradient's RMS (+1e-7:
    some gradients are analytically ~0, e.g. key biases under a row softmax), the L2 norm within
    rtol and the sum.  The floor covers fp32 summation: weight gradients are sums over 8k-32k
    frame rows whose terms cancel (the CPU fp32 oracle itself sits up to 1.4e-3 x RMS from fp64).
    Parameters whose name starts with a prefix in ``relaxed`` (see GruKinks: a ReLU sign flip
    between fp32 and fp64 right at the kink) are compared normwise: ||g - r|| <= relaxed_tol ||r||."""
    bad = []
    for n, p in net.named_parameters():
        g = p.grad
        assert g is not None, f"{what}{n}: no gradient"
        g = g.detach().double().cpu().reshape(-1).numpy()
        r = ref[n].detach().double().cpu().reshape(-1).numpy()
        rn = float(np.sqrt((r * r).sum()))
        if any(n.startswith(pre) for pre in relaxed):
            dn = float(np.sqrt(((g - r) ** 2).sum()))
            if dn > relaxed_tol * rn + 1e-7:
                bad.append(f"{n} (kink, normwise): |g - r| {dn:.3g} vs |r| {rn:.3g}")
            continue
        rms = float(np.sqrt((r * r).mean())) if r.size else 0.0
        idx = pg.sample_index(g.size)
        atol = atol_rms * rms + 1e-7
        err = np.abs(g[idx] - r[idx]) - (atol + rtol * np.abs(r[idx]))
        if (err > 0).any():
            bad.append(f"{n}: sample max excess {err.max():.3g} (rms {rms:.3g})")
            continue
        gn = float(np.sqrt((g * g).sum()))
        if abs(gn - rn) > rtol * rn + atol * np.sqrt(g.size):
            bad.append(f"{n}: norm {gn} vs {rn}")
        if abs(g.sum() - r.sum()) > rtol * rn * np.sqrt(g.size) + atol * g.size:
            bad.append(f"{n}: sum {g.sum()} vs {r.sum()}")
    assert not bad, what + "gradients differ:\n" + "\n".join(bad[:20])


class GruKinks:
    """Records the BiGRU outputs of the HIP path (factmx.functional.gru) and of the oracle
    (fact_oracle.gru) -- both feed ``relu(.)`` (blocks.py:432) -- so a test can tell where a ReLU
    sign differs between fp32 and fp64.  An output within ~1e-7 of 0 may round to the other side
    in fp32; the gradient of that ONE element is then dout vs 0 (a true discontinuity, not an
    error of either side) and it runs back through the recurrence into that block's GRU weight
    gradients.  ``flipped_prefixes`` names those blocks' seg_update parameters."""

    def __init__(self, monkeypatch):
        from factmx import functional as fxf
        from oracle import fact_oracle as fo
        self.gpu, self.ref = [], []
        g0, r0 = fxf.gru, fo.gru

        def gpu(mod, x, seq_off=None, relu=False):
            # (relu(y) > 0 exactly where y > 0: the sign test below reads either)
            y = g0(mod, x, seq_off=seq_off, relu=relu)
            self.gpu.append((y.detach(), seq_off))
            return y

        def ref(P, p, x, nl):
            y = r0(P, p, x, nl)
            self.ref.append((p, y.detach()))
            return y
        monkeypatch.setattr(fxf, "gru", gpu)
        monkeypatch.setattr(fo, "gru", ref)

    def flipped_prefixes(self, nvid):
        """Prefixes 'block_list.k.seg_update.' of the TDU blocks with a ReLU sign flip."""
        gpu_parts = []                          # per (video, U block), in video-major order
        lock = [c for c in self.gpu if c[1] is not None]
        if lock:
            nblk = len(lock)
            for v in range(nvid):
                for y, off in lock:
                    gpu_parts.append(y[off[v]:off[v + 1]])
        else:
            gpu_parts = [y for y, _ in self.gpu]
            nblk = len(gpu_parts) // max(nvid, 1)
        out = set()
        for i, (p, yr) in enumerate(self.ref[:len(gpu_parts)]):
            yg = gpu_parts[i].double().cpu()
            if ((yg > 0) != (yr > 0)).any():
                out.add(p)
        assert nblk * nvid == len(gpu_parts)
        return out


def drop_mask(seed, idx, p):
    """The kernels' dropout keep-mask (include/factmx.h fx_dropout): splitmix64 of
    seed + (idx + 1) * 0x9E3779B97F4A7C15, kept iff the high 32 bits >= p * 2^32 (p as float32)."""
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed % 2 ** 64) + (idx + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    bits = (z >> np.uint64(32)).astype(np.uint64)
    thr = min(int(float(np.float32(p)) * 4294967296.0), 4294967295)
    return bits >= np.uint64(max(thr, 1))


def drop_subseed(seed, i):
    """fx_drop_subseed: the seed of sub-site i (MS-TCN layer i) of a dropout site."""
    return (seed + 0xD1B54A32D192ED03 * (i + 1)) % 2 ** 64
