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
