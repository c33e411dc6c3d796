"""Seeded inputs for the evaluation-metric and dataset-reader fixtures (tests/golden/eval_io.npz).
Shared by make_eval_golden.py (reference side, build container) and tests/test_eval_io.py."""
import os

import numpy as np


def _runs(rng, T, ncls, nseg, bg=None):
    cuts = np.sort(rng.choice(np.arange(1, T), nseg - 1, replace=False))
    lens = np.diff(np.concatenate([[0], cuts, [T]]))
    labs = rng.integers(0, ncls, nseg)
    if bg is not None:
        labs[::3] = bg
    return np.repeat(labs, lens).astype(np.int64)


def eval_cases():
    rng = np.random.default_rng(11)
    c = {}
    c["same"] = (np.array([1, 1, 2, 2, 3]), np.array([1, 1, 2, 2, 3]), [0])
    c["single_vs_single"] = (np.full(50, 4), np.full(50, 4), [0])
    c["single_vs_many"] = (np.full(40, 2), np.repeat([1, 2, 3, 2], 10), [0])
    c["len1"] = (np.array([5]), np.array([5]), [0])
    c["len1_diff"] = (np.array([5]), np.array([6]), ["background"])
    c["alternating"] = (np.arange(30) % 2 + 1, np.repeat([1, 2], 15), [0])
    c["pred_all_bg"] = (np.zeros(20, np.int64), np.repeat([0, 3, 0, 4], 5), [0])
    c["both_all_bg"] = (np.zeros(12, np.int64), np.zeros(12, np.int64), [0])
    c["gt_all_bg"] = (np.repeat([0, 3], 6), np.zeros(12, np.int64), [0])
    for i in range(6):
        T = int(rng.integers(50, 3000))
        g = _runs(rng, T, 8, int(rng.integers(2, 25)), bg=0)
        p = _runs(rng, T, 8, int(rng.integers(2, 60)), bg=0)
        c[f"rand{i}"] = (p, g, [0] if i % 2 == 0 else ["background"])
    # near-identical boundaries: IoU around the thresholds
    g = np.repeat([1, 2, 3, 4], [100, 100, 100, 100])
    p = np.repeat([1, 2, 3, 4], [60, 130, 95, 115])
    c["shifted"] = (p, g, [0])
    return c


def checkpoint_cases():
    rng = np.random.default_rng(5)
    vids = []
    for k in range(4):
        T = int(rng.integers(200, 900))
        gt = _runs(rng, T, 9, int(rng.integers(3, 12)), bg=0)
        # prediction: gt with boundary jitter and some wrong labels, at half frame rate for two videos
        pr = gt.copy()
        pr[rng.integers(0, T, T // 10)] = rng.integers(0, 9, T // 10)
        if k % 2 == 1:
            pr = pr[::2].copy()
        vids.append((f"vid{k}", gt, pr))
    return {
        "plain": (vids, dict(bg_class=[0])),
        "nobg": (vids, dict(bg_class=[])),
        "holdout": (vids, dict(bg_class=[0], holdout_classes=[3, 5],
                               seen_classes=[c for c in range(9) if c not in (3, 5)])),
    }


def write_synthetic_dataset(root):
    """A HAViD-layout tree and a Breakfast-layout tree with 5 videos each under ``root``."""
    rng = np.random.default_rng(21)
    names = ["null", "pick screw", "place bolt", "insert gear", "turn knob", "grasp"]

    def tree(ds_root, feat_dir, bundle_suffix_txt, extra_line):
        os.makedirs(os.path.join(ds_root, "groundTruth"), exist_ok=True)
        os.makedirs(os.path.join(ds_root, "splits"), exist_ok=True)
        os.makedirs(feat_dir, exist_ok=True)
        with open(os.path.join(ds_root, "mapping.txt"), "w") as f:
            for i, n in enumerate(names):
                f.write(f"{i} {n}\n")
        vnames = [f"S{k:02d}_{'ab'[k % 2]}" for k in range(5)]
        for k, v in enumerate(vnames):
            T = int(rng.integers(40, 120))
            lab = _runs(rng, T, len(names), int(rng.integers(2, 6)), bg=0)
            if k == 1:
                lab[lab == 2] = 3          # video 1 never shows class 2 (kept under holdout [2])
            if k == 3:
                lab[5:9] = 2               # video 3 surely does
            with open(os.path.join(ds_root, "groundTruth", v + ".txt"), "w") as f:
                f.write("".join(names[c] + "\n" for c in lab))
            Tf = T + (3 if k == 2 else 0)   # one feature file longer than its labels (truncated)
            feat = rng.standard_normal((7, Tf)).astype(np.float64 if k == 0 else np.float32)
            np.save(os.path.join(feat_dir, v + ".npy"), feat)
        for split, vs in (("train", vnames[:4]), ("test", vnames[3:])):
            with open(os.path.join(ds_root, "splits", f"{split}.split1.bundle"), "w") as f:
                for v in vs:
                    f.write(v + (".txt" if bundle_suffix_txt else "") + "\n")
                if extra_line:
                    f.write("README.md\n")

    hb = os.path.join(root, "data/HAViD/ActionSegmentation/data")
    tree(os.path.join(hb, "view0_lh_pt"), os.path.join(hb, "features"), True, True)
    tree(os.path.join(root, "data/breakfast"), os.path.join(root, "data/breakfast/features"), True, False)


def dataset_cfgs():
    from factmx.configs import get_cfg_defaults
    out = {}
    for name, kw in {
        "havid": dict(dataset="havid_view0_lh_pt"),
        "havid_holdout_sr2": dict(dataset="havid_view0_lh_pt", holdout_mode=True, holdout_classes=[2], sr=2),
        "breakfast": dict(dataset="breakfast"),
    }.items():
        cfg = get_cfg_defaults()
        for k, v in kw.items():
            setattr(cfg, k, v)
        out[name] = cfg
    return out
