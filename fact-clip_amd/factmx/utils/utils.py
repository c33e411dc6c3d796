"""Host helpers with the reference's names (fact_clip/utils/utils.py)."""
import numpy as np
import torch

from ..models.basic import Segment  # noqa: F401  (same class name as utils.py:4)


def parse_label(label):
    """utils.py:25-48: run-length segments [start, end] (inclusive) of a label sequence."""
    label = np.asarray(label)
    change = np.nonzero(label[:-1] != label[1:])[0]
    starts = np.concatenate([[0], change + 1])
    ends = np.concatenate([change, [len(label) - 1]])
    return [Segment(label[s], int(s), int(e)) for s, e in zip(starts, ends)]


def to_numpy(x):
    """utils.py:133-140."""
    if isinstance(x, np.ndarray):
        return x
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


def expand_frame_label(label, target_len: int):
    """utils.py:52-74: nearest-neighbour resize of a (downsampled) label sequence back to
    ``target_len`` frames; the resize is torch's ``interpolate(mode="nearest")`` so the index
    rounding is the reference's exactly."""
    if len(label) == target_len:
        return label
    is_numpy = isinstance(label, np.ndarray)
    if is_numpy:
        t = torch.from_numpy(label).float()
    elif isinstance(label, list):
        t = torch.tensor(label, dtype=torch.float32)
    else:
        t = label
    out = torch.nn.functional.interpolate(t.reshape(1, 1, -1), size=target_len, mode="nearest").reshape(-1).long()
    return out.numpy() if is_numpy else out


def shrink_frame_label(label: list, clip_len: int) -> list:
    """utils.py:76-87: majority label of each ``clip_len`` window (ties -> the label seen first in
    the window, Counter.most_common order)."""
    out = []
    for s in range(0, len(label), clip_len):
        win = label[s:s + clip_len]
        counts = {}
        for v in win:
            counts[v] = counts.get(v, 0) + 1
        best = max(counts.values())
        out.append(next(v for v in counts if counts[v] == best))
    return out


def easy_reduce(scores, mode="mean", skip_nan=False):
    """utils.py:89-130: reduce a list of scalars / arrays / tuples / lists / dicts element-wise."""
    assert isinstance(scores, list), type(scores)
    if len(scores) == 0:
        return np.nan
    first = scores[0]
    if isinstance(first, list):
        return [easy_reduce([s[i] for s in scores], mode=mode, skip_nan=skip_nan) for i in range(len(first))]
    if isinstance(first, np.ndarray):
        assert first.ndim == 1
        return np.stack(scores, axis=0).mean(0)
    if isinstance(first, tuple):
        return tuple(easy_reduce([s[i] for s in scores], mode=mode, skip_nan=skip_nan) for i in range(len(first)))
    if isinstance(first, dict):
        return {k: easy_reduce([s[k] for s in scores], mode=mode, skip_nan=skip_nan) for k in first}
    if isinstance(first, (float, int, np.float32)):
        if skip_nan:
            scores = [x for x in scores if not np.isnan(x)]
        if mode == "mean":
            return np.mean(scores)
        if mode == "max":
            return np.max(scores)
        if mode == "median":
            return np.median(scores)
        return None
    raise TypeError("Unsupport Data Type %s" % type(first))
