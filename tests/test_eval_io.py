"""Evaluation metrics and dataset readers vs the reference's outputs.

Fixtures: tests/golden/eval_io.npz, captured from the reference by
tests/golden/make_eval_golden.py on the seeded inputs of tests/golden/eval_cases.py.
Integer results (labels, video lists, counts) are compared exactly; metric values
(Edit, F1, accuracies) to 1e-12 relative (same float64 arithmetic, different order).
"""
import json
import os

import numpy as np
import pytest
import torch

from eval_cases import checkpoint_cases, dataset_cfgs, eval_cases, write_synthetic_dataset
from factmx.utils import dataset as ds
from factmx.utils import evaluate as ev
from factmx.utils.utils import easy_reduce, expand_frame_label, parse_label, shrink_frame_label
from helpers import load_fixture


@pytest.fixture(scope="module")
def fx():
    return load_fixture("eval_io")


def test_levenshtein_edit_f1(fx):
    for name, (p, y, bg) in eval_cases().items():
        ps, ys = parse_label(p), parse_label(y)
        got = np.array([ev.levenstein(p, y), ev.levenstein(p, y, norm=True)])
        np.testing.assert_allclose(got, fx[f"lev/{name}"], rtol=1e-12, equal_nan=True, err_msg=name)
        np.testing.assert_allclose([ev.edit_score(ps, ys, bg_class=bg)], fx[f"edit/{name}"], rtol=1e-12,
                                   equal_nan=True, err_msg=name)
        want = fx[f"f1/{name}"]
        if want.shape == (1,) and want[0] == -1.0:
            with pytest.raises(ValueError):
                ev.f_score(ps, ys, 0.1, bg_class=bg)
        else:
            got = np.array([ev.f_score(ps, ys, ov, bg_class=bg) for ov in (0.1, 0.25, 0.5)])
            np.testing.assert_array_equal(got, want, err_msg=name)


def test_checkpoint_metrics(fx, tmp_path):
    for name, (videos, kw) in checkpoint_cases().items():
        ck = ev.Checkpoint(0, **kw)
        ck.add_videos([ev.Video(vn, gt_label=gt, pred=pr) for vn, gt, pr in videos])
        m = ck.compute_metrics()
        assert list(m.keys()) == list(fx[f"ckpt/{name}/keys"]), name
        np.testing.assert_allclose([float(v) for v in m.values()], fx[f"ckpt/{name}/values"], rtol=1e-12)
        pc = ck.per_class_metrics
        np.testing.assert_array_equal([[c, pc[c]["correct"], pc[c]["total"]] for c in sorted(pc)],
                                      fx[f"ckpt/{name}/per_class"])
        np.testing.assert_array_equal(np.concatenate([v.pred_label for v in ck.videos.values()]),
                                      fx[f"ckpt/{name}/pred_label"])
    # persistence round trips
    ck.save(str(tmp_path / "ck.gz"))
    assert ev.Checkpoint.load(str(tmp_path / "ck.gz")).metrics.keys() == ck.metrics.keys()
    ck.save_detailed_results(str(tmp_path / "res.json"))
    res = json.load(open(tmp_path / "res.json"))
    assert set(res["per_video_results"]) == {"vid0", "vid1", "vid2", "vid3"}


def test_label_helpers(fx):
    rng = np.random.default_rng(7)
    lab = list(rng.integers(0, 4, 103))
    for sr in (2, 3, 8):
        np.testing.assert_array_equal(shrink_frame_label(lab, sr), fx[f"shrink/{sr}"])
    small = rng.integers(0, 9, 37)
    for tl in (37, 50, 111, 300, 1001):
        np.testing.assert_array_equal(expand_frame_label(small, tl), fx[f"expand/{tl}"])
    got = easy_reduce([{"a": 1.0, "b": np.nan}, {"a": 2.0, "b": 4.0}, {"a": 4.5, "b": 1.0}], skip_nan=True)
    np.testing.assert_allclose(list(got.values()), fx["reduce/dict"])


def test_create_dataset(fx, tmp_path):
    write_synthetic_dataset(str(tmp_path))
    for name, cfg in dataset_cfgs().items():
        tr, te = ds.create_dataset(cfg, base=str(tmp_path))
        for tag, d in (("train", tr), ("test", te)):
            p = f"ds/{name}/{tag}"
            assert d.get_vnames() == list(fx[f"{p}/videos"])
            np.testing.assert_allclose([d.nclasses, d.input_dimension, d.average_transcript_len], fx[f"{p}/meta"])
            np.testing.assert_array_equal(d.seen_classes, fx[f"{p}/seen"])
            np.testing.assert_array_equal(np.array(d.holdout_classes, dtype=np.int64), fx[f"{p}/holdout"])
            for v in d.get_vnames():
                f, tl, el = d[v]
                assert f.dtype == np.float32
                np.testing.assert_array_equal(f.shape, fx[f"{p}/{v}/feat_shape"])
                np.testing.assert_array_equal([f.astype(np.float64).sum(), f[0, 0], f[-1, -1]],
                                              fx[f"{p}/{v}/feat_sum"])
                np.testing.assert_array_equal(tl, fx[f"{p}/{v}/train_label"])
                np.testing.assert_array_equal(el, fx[f"{p}/{v}/eval_label"])
        np.random.seed(3)
        dl = ds.DataLoader(tr, 2, shuffle=True)
        order = []
        for _ in range(2):
            for names, seqs, labs, evs in dl:
                assert all(s.dtype == torch.float32 for s in seqs) and all(l.dtype == torch.long for l in labs)
                order.extend(names)
        assert order == list(fx[f"ds/{name}/loader_order"])
    l2i, i2l = ds.load_action_mapping(str(tmp_path / "data/HAViD/ActionSegmentation/data/view0_lh_pt/mapping.txt"))
    assert json.dumps(l2i, sort_keys=True) == str(fx["ds/mapping"])
    assert all(l2i[i2l[i]] == i for i in i2l)


def test_holdout_filter_unreadable(tmp_path, capsys):
    assert ds.video_contains_holdout_classes("missing", str(tmp_path), {}, [1]) is False
    assert "Warning" in capsys.readouterr().out


@pytest.mark.gpu
def test_device_prefetcher_matches_loader(tmp_path):
    write_synthetic_dataset(str(tmp_path))
    cfg = dataset_cfgs()["havid"]
    tr, _ = ds.create_dataset(cfg, base=str(tmp_path))
    want = [(n, [s.clone() for s in q], [l.clone() for l in b]) for n, q, b, _ in ds.DataLoader(tr, 2)]
    got = list(ds.DevicePrefetcher(ds.DataLoader(tr, 2), "cuda"))
    assert len(got) == len(want)
    for (n0, q0, b0), (n1, q1, b1, _) in zip(want, got):
        assert n0 == n1
        for a, b in zip(q0 + b0, q1 + b1):
            assert b.is_cuda
            assert torch.equal(a, b.cpu())
