"""The fused loss phase of a lockstep batch (models/vloss.py: fx_eval_pred, fx_match_cost,
fx_loss_terms_fwd/bwd) against the per-video MatchCriterion path on the same forward (GPU):
predictions and matchings identical, batch loss and every per-video loss value within fp32
summation-order tolerance, every parameter gradient within 1e-4 of its max.  Cases: the tiny
golden config, the benchmark shape (T=4096, 2 videos), held-out classes inside the labels (masked
InfoNCE rows, one video fully held out), one-to-many matching, background class weights."""
import numpy as np
import pytest
import torch

import paramgen as pg
from helpers import load_fixture, tiny_meta, cfg_from_meta, tiny_inputs
from factmx.models import blocks as blocks_mod
from factmx.models import loss as loss_mod

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tiny(name="tiny_clip", bg_ids=()):
    from factmx.models.blocks import FACT_CLIP
    fx = load_fixture(name)
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    C, D = meta["C"], meta["D"]
    feats, label, text = tiny_inputs(meta)
    net = FACT_CLIP(cfg, D, C, text_embeddings=torch.from_numpy(text).float())
    with torch.no_grad():
        for n, p in net.named_parameters():
            p.copy_(torch.from_numpy(pg.param_value(n, p.shape, meta["seed"])))
    net.mcriterion = loss_mod.MatchCriterion(cfg, C, list(bg_ids))
    return net.to(DEV).train(), cfg, meta, feats, label


def _run(net, seqs, labs, fused, monkeypatch):
    monkeypatch.setattr(blocks_mod, "FUSED_LOSS", fused)
    for k in ("fact_loss", "contrastive_loss"):       # both runs start from the same side channels
        net.__dict__.pop(k, None)
    net.zero_grad(set_to_none=True)
    total, saves = net(seqs, labs, compute_loss=True)
    total.backward()
    torch.cuda.synchronize()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters() if p.grad is not None}
    return total.item(), saves, grads


def _compare(net, seqs, labs, monkeypatch, loss_tol=2e-5, grad_tol=1e-4):
    ref = _run(net, seqs, labs, False, monkeypatch)
    got = _run(net, seqs, labs, True, monkeypatch)
    assert abs(got[0] - ref[0]) <= loss_tol * max(1.0, abs(ref[0])), (got[0], ref[0])
    for v, (a, b) in enumerate(zip(got[1], ref[1])):
        np.testing.assert_array_equal(a["pred"], b["pred"], err_msg=f"video {v}")
        assert sorted(a["loss"]) == sorted(b["loss"]), (a["loss"], b["loss"])
        for k in b["loss"]:
            assert abs(a["loss"][k] - b["loss"][k]) <= loss_tol * max(1.0, abs(b["loss"][k])), (v, k, a["loss"],
                                                                                               b["loss"])
    assert sorted(got[2]) == sorted(ref[2])
    for n, g in ref[2].items():
        err = (got[2][n] - g).abs().max().item()
        assert err <= grad_tol * g.abs().max().item() + 1e-7, (n, err, g.abs().max().item())
    return got


def _two_videos(meta, feats, label, seed=11):
    T, D = feats.shape
    seen = sorted(set(label.tolist()))
    f2, l2 = pg.segmented_video(T, D, seen, 5, seed=seed, noise=0.4)
    seqs = [torch.from_numpy(feats).float().to(DEV), torch.from_numpy(f2).float().to(DEV)]
    labs = [torch.from_numpy(label).to(DEV), torch.from_numpy(l2).to(DEV)]
    return seqs, labs


@pytest.mark.parametrize("name", ["tiny_clip", "tiny_clip_iid"])
def test_fused_loss_equals_per_video_tiny(name, monkeypatch):
    net, cfg, meta, feats, label = _tiny(name)
    seqs, labs = _two_videos(meta, feats, label)
    assert blocks_mod._batchable(net, seqs) and blocks_mod.vloss.supported(net)
    _compare(net, seqs, labs, monkeypatch)


def test_fused_loss_background_weights_and_o2m(monkeypatch):
    label = _tiny("tiny_clip")[4]
    net, cfg, meta, feats, label = _tiny("tiny_clip", bg_ids=(int(label[0]),))
    cfg.Loss.bgw = 0.3
    seqs, labs = _two_videos(meta, feats, label, seed=5)
    _compare(net, seqs, labs, monkeypatch)
    cfg.Loss.match = "o2m"
    _compare(net, seqs, labs, monkeypatch)


def test_fused_loss_holdout_rows_masked(monkeypatch):
    net, cfg, meta, feats, label = _tiny("tiny_clip")
    T = feats.shape[0]
    C = meta["C"]
    hold = [c for c in range(C) if c not in set(label.tolist())][:3]
    cfg.holdout_classes = hold
    cfg.holdout_mode = True
    seqs, labs = _two_videos(meta, feats, label)
    l0 = labs[0].clone()
    l0[T // 3: T // 2] = hold[0]              # some frames of video 0 carry a held-out class
    l1 = torch.full_like(labs[1], hold[1])    # video 1 entirely held out: fact loss only
    _compare(net, seqs, [l0, l1], monkeypatch)


def test_fused_loss_north_star_shape(monkeypatch):
    from bench import make_cfg, make_video, build_model as bench_model
    cfg = make_cfg()
    T, D, C = 4096, 2048, 75
    net, _ = bench_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
    seqs = [torch.from_numpy(f).to(DEV) for f, _ in vids]
    labs = [torch.from_numpy(l_).to(DEV) for _, l_ in vids]
    assert blocks_mod.vloss.supported(net)
    _compare(net, seqs, labs, monkeypatch, grad_tol=2e-4)


def test_fused_eval_only(monkeypatch):
    net, cfg, meta, feats, label = _tiny("tiny_clip")
    seqs, labs = _two_videos(meta, feats, label)
    with torch.no_grad():
        monkeypatch.setattr(blocks_mod, "FUSED_LOSS", False)
        ref = net(seqs, labs, compute_loss=False)
        monkeypatch.setattr(blocks_mod, "FUSED_LOSS", True)
        got = net(seqs, labs, compute_loss=False)
    for a, b in zip(got, ref):
        np.testing.assert_array_equal(a["pred"], b["pred"])
