"""Capture golden vectors for the evaluation metrics and dataset readers from the reference
(build container only; nothing here ships or runs on the GPU box).

Run:  python tests/golden/make_eval_golden.py   -> tests/golden/eval_io.npz

Inputs are regenerated from seeds by ``eval_cases()`` / ``write_synthetic_dataset()`` (shared
with tests/test_eval_io.py); the fixture stores only the reference's outputs:
  * levenstein / edit_score / f_score on label-sequence pairs (edge cases + random);
  * Checkpoint.compute_metrics (plain and holdout mode, with a downsampled prediction that goes
    through expand_frame_label);
  * shrink_frame_label / expand_frame_label / easy_reduce;
  * create_dataset on a synthetic HAViD-layout tree (mapping, groundTruth, (D,T) .npy features,
    bundles, holdout filtering, sr=2) written to a temp dir; the reference's module global
    ``BASE`` is pointed at it.
"""
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
sys.path.insert(0, os.path.join(HERE, "_yacs_shim"))
sys.path.insert(0, REF)
sys.path.insert(0, HERE)

from eval_cases import eval_cases, checkpoint_cases, write_synthetic_dataset, dataset_cfgs  # noqa: E402
from fact_clip.utils import evaluate as rev  # noqa: E402
from fact_clip.utils import utils as rut  # noqa: E402
from fact_clip.utils import dataset as rds  # noqa: E402


def main():
    out = {}
    for name, (p, y, bg) in eval_cases().items():
        ps, ys = rut.parse_label(p), rut.parse_label(y)
        out[f"lev/{name}"] = np.array([rev.levenstein(p, y), rev.levenstein(p, y, norm=True)])
        out[f"edit/{name}"] = np.array([rev.edit_score(ps, ys, bg_class=bg)])
        try:
            out[f"f1/{name}"] = np.array([rev.f_score(ps, ys, ov, bg_class=bg) for ov in (0.1, 0.25, 0.5)])
        except ValueError:
            out[f"f1/{name}"] = np.array([-1.0])   # reference raises (no foreground ground truth)

    for name, (videos, kw) in checkpoint_cases().items():
        ck = rev.Checkpoint(0, **kw)
        ck.add_videos([rev.Video(vn, gt_label=gt, pred=pr) for vn, gt, pr in videos])
        m = ck.compute_metrics()
        out[f"ckpt/{name}/keys"] = np.array(list(m.keys()))
        out[f"ckpt/{name}/values"] = np.array([float(v) for v in m.values()])
        pc = ck.per_class_metrics
        out[f"ckpt/{name}/per_class"] = np.array([[c, pc[c]["correct"], pc[c]["total"]] for c in sorted(pc)])
        out[f"ckpt/{name}/pred_label"] = np.concatenate([v.pred_label for v in ck.videos.values()])

    rng = np.random.default_rng(7)
    lab = list(rng.integers(0, 4, 103))
    for sr in (2, 3, 8):
        out[f"shrink/{sr}"] = np.array(rut.shrink_frame_label(lab, sr))
    small = rng.integers(0, 9, 37)
    for tl in (37, 50, 111, 300, 1001):
        out[f"expand/{tl}"] = np.asarray(rut.expand_frame_label(small, tl))
    out["reduce/dict"] = np.array(list(rut.easy_reduce(
        [{"a": 1.0, "b": np.nan}, {"a": 2.0, "b": 4.0}, {"a": 4.5, "b": 1.0}], skip_nan=True).values()))

    with tempfile.TemporaryDirectory() as tmp:
        write_synthetic_dataset(tmp)
        rds.BASE = tmp + "/"
        for name, cfg in dataset_cfgs().items():
            tr, te = rds.create_dataset(cfg)
            for tag, d in (("train", tr), ("test", te)):
                out[f"ds/{name}/{tag}/videos"] = np.array(d.get_vnames())
                out[f"ds/{name}/{tag}/meta"] = np.array([d.nclasses, d.input_dimension, d.average_transcript_len])
                out[f"ds/{name}/{tag}/seen"] = np.array(d.seen_classes)
                out[f"ds/{name}/{tag}/holdout"] = np.array(d.holdout_classes, dtype=np.int64)
                for v in d.get_vnames():
                    f, tl, el = d[v]
                    out[f"ds/{name}/{tag}/{v}/feat_shape"] = np.array(f.shape)
                    out[f"ds/{name}/{tag}/{v}/feat_sum"] = np.array([f.astype(np.float64).sum(), f[0, 0], f[-1, -1]])
                    out[f"ds/{name}/{tag}/{v}/train_label"] = np.array(tl)
                    out[f"ds/{name}/{tag}/{v}/eval_label"] = np.array(el)
            # DataLoader order with a fixed numpy seed
            np.random.seed(3)
            dl = rds.DataLoader(tr, 2, shuffle=True)
            order = []
            for _ in range(2):
                for names, seqs, labs, evs in dl:
                    order.extend(names)
            out[f"ds/{name}/loader_order"] = np.array(order)
        l2i, _ = rds.load_action_mapping(os.path.join(tmp, "data/HAViD/ActionSegmentation/data/view0_lh_pt/mapping.txt"))
        out["ds/mapping"] = np.array(json.dumps(l2i, sort_keys=True))

    np.savez_compressed(os.path.join(HERE, "eval_io.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    main()
