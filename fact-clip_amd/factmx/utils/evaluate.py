"""Segmentation metrics with the reference's names and results
(fact_clip/utils/evaluate.py): framewise accuracy (with / without background),
segmental Edit score, F1@{0.10,0.25,0.50}, per-class accuracy and the holdout
seen/unseen split.

The arithmetic is restated with numpy: the Levenshtein table is filled one row
at a time (the left-neighbour dependency is a running minimum), and the F1
overlap matrix is computed for all (pred, gt) segment pairs at once before the
greedy first-come matching the reference does. Results are identical to the
reference's (tests/test_eval_io.py against tests/golden/eval_io.npz, captured
from the reference by tests/golden/make_eval_golden.py).
"""
import gzip
import json
import pickle
from collections import OrderedDict

import numpy as np

from .utils import easy_reduce, expand_frame_label, parse_label

OVERLAPS = (0.1, 0.25, 0.5)


def levenstein(p, y, norm=False):
    """evaluate.py:7-30 — edit distance between two label sequences; with ``norm`` the score
    ``(1 - d / max(len)) * 100``."""
    p = np.asarray(p)
    y = np.asarray(y)
    m, n = len(p), len(y)
    cols = np.arange(n + 1, dtype=np.float64)
    prev = cols.copy()                                   # row 0: D[0, j] = j
    for i in range(1, m + 1):
        diag = prev[:-1] + (y != p[i - 1])               # substitute / match
        up = prev[1:] + 1.0                              # delete
        cand = np.empty(n + 1)
        cand[0] = i
        cand[1:] = np.minimum(diag, up)
        # insertion: D[i, j] = min_k<=j (cand[k] + j - k)
        prev = np.minimum.accumulate(cand - cols) + cols
    d = np.float64(prev[-1])
    if norm:
        with np.errstate(invalid="ignore", divide="ignore"):
            return (1 - d / np.float64(max(m, n))) * 100      # NaN for two empty sequences, as numpy gives
    return d


def segs_to_labels_start_end_time(seg_list, bg_class):
    """evaluate.py:32-37 — foreground segments as (labels, starts, exclusive ends)."""
    seg_list = [s for s in seg_list if s.action not in bg_class]
    return ([s.action for s in seg_list], [s.start for s in seg_list], [s.end + 1 for s in seg_list])


def edit_score(pred_segs, gt_segs, norm=True, bg_class=["background"]):
    """evaluate.py:39-42."""
    P, _, _ = segs_to_labels_start_end_time(pred_segs, bg_class)
    Y, _, _ = segs_to_labels_start_end_time(gt_segs, bg_class)
    return levenstein(P, Y, norm)


def f_score(pred_segs, gt_segs, overlap, bg_class=["background"]):
    """evaluate.py:44-67 — greedy matching of predicted to ground-truth segments at an IoU
    threshold; returns (tp, fp, fn) as floats."""
    pl, ps, pe = (np.asarray(v) for v in segs_to_labels_start_end_time(pred_segs, bg_class))
    yl, ys, ye = (np.asarray(v) for v in segs_to_labels_start_end_time(gt_segs, bg_class))
    if len(pl) == 0:
        return 0.0, 0.0, float(len(yl))
    inter = np.minimum(pe[:, None], ye[None, :]) - np.maximum(ps[:, None], ys[None, :])
    union = np.maximum(pe[:, None], ye[None, :]) - np.minimum(ps[:, None], ys[None, :])
    iou = (1.0 * inter / union) * (pl[:, None] == yl[None, :])
    best = iou.argmax(axis=1)                            # raises on empty gt, as the reference
    hits = np.zeros(len(yl), dtype=bool)
    tp = fp = 0
    for j in range(len(pl)):
        idx = best[j]
        if iou[j, idx] >= overlap and not hits[idx]:
            tp += 1
            hits[idx] = True
        else:
            fp += 1
    return float(tp), float(fp), float(len(yl) - hits.sum())


def _member(x, values):
    """Per-element ``x[i] in values`` (the reference's list comprehension), vectorised for numbers."""
    values = list(values)
    if all(isinstance(v, (int, np.integer)) for v in values) and np.issubdtype(x.dtype, np.integer):
        return np.isin(x, np.asarray(values, dtype=np.int64))
    return np.array([g in values for g in x], dtype=bool)


def _f1(tp, fp, fn):
    precision = tp / float(tp + fp + 1e-5)
    recall = tp / float(tp + fn + 1e-5)
    return np.nan_to_num(2.0 * (precision * recall) / (precision + recall + 1e-5)) * 100


class Video:
    """evaluate.py:70-81 — attribute bag for one evaluated video."""

    def __init__(self, vname="", **kwargs):
        self.vname = vname
        for k, v in kwargs.items():
            setattr(self, k, v)

    def __str__(self):
        return "< Video %s >" % self.vname

    __repr__ = __str__


class Checkpoint:
    """evaluate.py:83-271 — collects per-video predictions of one iteration and computes the
    joint metrics (same keys, same values)."""

    def __init__(self, iteration, bg_class=[], eval_edit=True, holdout_classes=[], seen_classes=None):
        self.iteration = iteration
        self.videos = {}
        self.bg_class = bg_class
        self.eval_edit = eval_edit
        self.holdout_classes = holdout_classes if holdout_classes is not None else []
        self.seen_classes = seen_classes if seen_classes is not None else []
        self.per_class_metrics = {}

    def add_videos(self, videos):
        for v in videos:
            self.videos[v.vname] = v

    # evaluate.py:104-115: gzip-pickled checkpoint files (written by this class only)
    @staticmethod
    def load(fname):
        with gzip.open(fname, "rb") as fp:
            return pickle.load(fp)

    def save(self, fname):
        self.fname = fname
        with gzip.open(fname, "wb") as fp:
            pickle.dump(self, fp)

    def __str__(self):
        return "< Checkpoint[%d] %d videos >" % (self.iteration, len(self.videos))

    __repr__ = __str__

    def _random_video(self):
        vname = np.random.choice(list(self.videos.keys()), 1).item()
        return vname, self.videos[vname]

    def average_losses(self):
        self.loss = easy_reduce([v.loss for v in self.videos.values()], mode="mean")

    def _per_video_metrics(self, gt_label, pred_label):
        M = OrderedDict()
        if self.eval_edit:
            M["Edit"] = edit_score(parse_label(pred_label), parse_label(gt_label), bg_class=self.bg_class)
        return M

    @staticmethod
    def _f1_counts(pairs, bg_class):
        tp, fp, fn = np.zeros(3), np.zeros(3), np.zeros(3)
        for pred_segs, gt_segs in pairs:
            for s, ov in enumerate(OVERLAPS):
                a, b, c = f_score(pred_segs, gt_segs, ov, bg_class=bg_class)
                tp[s] += a
                fp[s] += b
                fn[s] += c
        return tp, fp, fn

    def _joint_metrics(self, gt_list, pred_list):
        M = OrderedDict()
        gt_ = np.concatenate(gt_list)
        pred_ = np.concatenate(pred_list)
        correct = gt_ == pred_
        fg_loc = ~_member(gt_, self.bg_class)
        M["AccB"] = correct.mean() * 100
        M["Acc"] = correct[fg_loc].mean() * 100

        segs = [(parse_label(p), parse_label(g)) for g, p in zip(gt_list, pred_list)]
        tp, fp, fn = self._f1_counts(segs, self.bg_class)
        for s, ov in enumerate(OVERLAPS):
            M["F1@%0.2f" % ov] = _f1(tp[s], fp[s], fn[s])

        classes, totals = np.unique(gt_, return_counts=True)
        for cls, tot in zip(classes, totals):
            ok = int(correct[gt_ == cls].sum())
            self.per_class_metrics[int(cls)] = {"correct": ok, "total": int(tot),
                                                "accuracy": float(ok / tot * 100)}

        if len(self.holdout_classes) > 0:
            for tag, cls_list in (("seen", self.seen_classes), ("unseen", self.holdout_classes)):
                mask = _member(gt_, cls_list)
                if mask.sum() > 0:
                    M[f"Acc-{tag}"] = correct[mask].mean() * 100
                    fgm = mask & fg_loc
                    if fgm.sum() > 0:
                        M[f"AccFG-{tag}"] = correct[fgm].mean() * 100
            for tag, cls_list in (("seen", self.seen_classes), ("unseen", self.holdout_classes)):
                pairs = []
                for ps, gs in segs:
                    gk = [s for s in gs if s.action in cls_list]
                    if len(gk) > 0:
                        pairs.append(([s for s in ps if s.action in cls_list], gk))
                tp, fp, fn = self._f1_counts(pairs, self.bg_class)
                for s, ov in enumerate(OVERLAPS):
                    if tp[s] + fp[s] + fn[s] > 0:
                        M[f"F1@{ov:.2f}-{tag}"] = _f1(tp[s], fp[s], fn[s])
        return M

    def compute_metrics(self):
        gt_list, pred_list = [], []
        for video in self.videos.values():
            video.pred_label = expand_frame_label(video.pred, len(video.gt_label))
            video.metrics = self._per_video_metrics(video.gt_label, video.pred_label)
            gt_list.append(video.gt_label)
            pred_list.append(video.pred_label)
        self.metrics = easy_reduce([v.metrics for v in self.videos.values()], skip_nan=True)
        self.metrics.update(self._joint_metrics(gt_list, pred_list))
        return self.metrics

    def save_detailed_results(self, fname):
        """evaluate.py:243-271 — metrics, per-class and per-video results as JSON."""
        def _list(x):
            return x.tolist() if hasattr(x, "tolist") else list(x)
        results = {
            "iteration": self.iteration,
            "metrics": {k: float(v) for k, v in dict(self.metrics).items()},
            "per_class_metrics": self.per_class_metrics,
            "holdout_classes": list(self.holdout_classes),
            "seen_classes": list(self.seen_classes),
            "per_video_results": {
                vname: {"gt_label": _list(v.gt_label), "pred_label": _list(v.pred_label),
                        "metrics": {k: float(x) for k, x in getattr(v, "metrics", {}).items()}}
                for vname, v in self.videos.items()},
        }
        with open(fname, "w") as f:
            json.dump(results, f, indent=2)
        print(f"Detailed results saved to: {fname}")
