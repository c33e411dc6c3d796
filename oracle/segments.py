"""Integer segmentation restated in numpy (oracle; test infrastructure only).

Follows the reference semantics exactly; every function cites the file:line it
restates.  Vectorised (no per-frame Python loop) but bit-identical in output.
"""
import numpy as np


def run_length_segments(label):
    """Restates ``parse_label`` (fact_clip/utils/utils.py:25-48).

    Returns int64 arrays ``(action, start, end)`` with inclusive ``end``:
    a new segment starts wherever ``label[t] != label[t-1]``.
    """
    label = np.asarray(label)
    n = label.shape[0]
    if n == 0:
        raise ValueError("empty label sequence")
    change = np.nonzero(label[:-1] != label[1:])[0]          # utils.py:29-30
    starts = np.concatenate([[0], change + 1]).astype(np.int64)
    ends = np.concatenate([change, [n - 1]]).astype(np.int64)
    return label[starts].astype(np.int64), starts, ends


def transcript_and_segment_ids(label):
    """Restates ``torch_class_label_to_segment_label`` (basic.py:38-54, dup loss.py:20-36).

    transcript = class of each run; seg_id[t] = index of the run frame t is in.
    """
    label = np.asarray(label)
    if label.shape[0] == 0:
        raise ValueError("empty label sequence")
    change = np.concatenate([[False], label[1:] != label[:-1]])
    seg_id = np.cumsum(change).astype(np.int64)
    transcript = label[np.concatenate([[True], change[1:]])].astype(np.int64)
    return transcript, seg_id


def segment_ids_from_bounds(starts, ends, n):
    """``TemporalDownsampleUpsample.seg_label`` (basic.py:601-605): frame -> segment id."""
    seg = np.empty(n, dtype=np.int64)
    for i, (s, e) in enumerate(zip(starts, ends)):
        seg[s:e + 1] = i
    return seg


def segment_centers(starts, ends):
    """``int((s.start+s.end)/2)`` (blocks.py:454) for non-negative ints == floor division."""
    return ((np.asarray(starts) + np.asarray(ends)) // 2).astype(np.int64)
