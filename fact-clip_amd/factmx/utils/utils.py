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
