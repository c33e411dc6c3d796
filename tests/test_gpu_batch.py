"""Lockstep multi-video path (blocks._forward_videos -> _FACTBase._forward_batch) vs the reference's
one-video-at-a-time loop on the same model and inputs (GPU; FACT_CLIP, and vanilla FACT with the
MS-TCN++ 'm2' frame branch of the Breakfast config): per-video predictions and TDU segment
boundaries identical, per-video losses / the batch loss and every parameter gradient within fp32
tolerance, the side-channel attributes (last video) equal; the first video also against the
reference golden vectors, and at the benchmark shape both videos against the CPU oracle."""
import numpy as np
import pytest
import torch

import paramgen as pg
from helpers import load_fixture, tiny_meta, cfg_from_meta, tiny_inputs
from oracle import fact_oracle as fo
from factmx.models import blocks as blocks_mod

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(meta, cfg):
    from factmx.models.blocks import FACT, FACT_CLIP
    from factmx.models.loss import MatchCriterion
    C, D = meta["C"], meta["D"]
    _, _, text = tiny_inputs(meta)
    if meta["model"] == "FACT_CLIP":
        net = FACT_CLIP(cfg, D, C, text_embeddings=torch.from_numpy(text).float())
    else:
        net = FACT(cfg, D, C)
    with torch.no_grad():
        for n, p in net.named_parameters():
            p.copy_(torch.from_numpy(pg.param_value(n, p.shape, meta["seed"])))
    net.mcriterion = MatchCriterion(cfg, C, [])
    return net.to(DEV).train()


def _run(net, seqs, labs, batched, monkeypatch):
    if not batched:
        monkeypatch.setattr(blocks_mod, "_batchable", lambda *a: False)
    else:
        monkeypatch.setattr(blocks_mod, "_batchable", blocks_mod.__dict__["_batchable_impl"])
    total, saves = net(seqs, labs, compute_loss=True)
    total.backward()
    torch.cuda.synchronize()
    attrs = {}
    for i, blk in enumerate(net.block_list):
        attrs[f"{i}/frame_clogit"] = blk.frame_clogit.detach().clone()
        attrs[f"{i}/action_clogit"] = blk.action_clogit.detach().clone()
        if hasattr(blk, "a2f_attn"):
            attrs[f"{i}/a2f_attn"] = blk.a2f_attn.detach().clone()
            attrs[f"{i}/f2a_attn_logit"] = blk.f2a_attn_logit.detach().clone()
        if hasattr(blk, "tdu"):
            attrs[f"{i}/seg_start"] = blk.tdu.start32.cpu().clone()
    if hasattr(net, "projected_frame_embeddings"):
        attrs["proj"] = net.projected_frame_embeddings.detach().clone()
    grads = {n: p.grad.detach().clone() for n, p in net.named_parameters()}
    return total.item(), saves, attrs, grads


@pytest.fixture(autouse=True)
def _keep_impl():
    blocks_mod.__dict__.setdefault("_batchable_impl", blocks_mod._batchable)
    yield


@pytest.mark.parametrize("name,dT", [("tiny_clip", 0), ("tiny_clip_iid", 0), ("tiny_fact_m2", 0),
                                     ("tiny_clip", -37), ("tiny_clip_iid", 23), ("tiny_fact_m2", -61)])
def test_lockstep_equals_per_video(name, dT, monkeypatch):
    """dT != 0: a ragged batch (the second video dT frames longer / shorter), as the reference's
    DataLoader yields (dataset.py:106-131)."""
    fx = load_fixture(name)
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    feats, label, _ = tiny_inputs(meta)
    T, D = feats.shape
    seen = sorted(set(label.tolist()))
    f2, l2 = pg.segmented_video(T + dT, D, seen, 5, seed=11, noise=0.4)
    seqs = [torch.from_numpy(feats).float().to(DEV), torch.from_numpy(f2).float().to(DEV)]
    labs = [torch.from_numpy(label).to(DEV), torch.from_numpy(l2).to(DEV)]
    assert blocks_mod._batchable(_model(meta, cfg), seqs)
    ref = _run(_model(meta, cfg), seqs, labs, False, monkeypatch)
    got = _run(_model(meta, cfg), seqs, labs, True, monkeypatch)
    assert abs(got[0] - ref[0]) <= 2e-5 * max(1.0, abs(ref[0]))
    for a, b in zip(got[1], ref[1]):
        np.testing.assert_array_equal(a["pred"], b["pred"])
        for k in b["loss"]:
            assert abs(a["loss"][k] - b["loss"][k]) <= 2e-5 * max(1.0, abs(b["loss"][k])), k
    for k, v in ref[2].items():
        if k.endswith("seg_start"):
            np.testing.assert_array_equal(got[2][k].numpy(), v.numpy(), err_msg=k)
        else:
            err = (got[2][k] - v).abs().max().item()
            assert err <= 1e-4 * max(1.0, v.abs().max().item()), (k, err)
    for n, g in ref[3].items():
        err = (got[3][n] - g).abs().max().item()
        assert err <= 1e-3 * g.abs().max().item() + 1e-6, (n, err)
    # the first video is the golden one: its prediction and loss match the reference capture
    np.testing.assert_array_equal(got[1][0]["pred"], fx["pred"])
    np.testing.assert_allclose(got[1][0]["loss"]["loss"], fx["loss"][0], rtol=2e-5)


def test_lockstep_north_star_vs_oracle():
    from bench import make_cfg, make_video, build_model as bench_model
    cfg = make_cfg()
    T, D, C = 4096, 2048, 75
    net, text = bench_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
    seqs = [torch.from_numpy(f).to(DEV) for f, _ in vids]
    labs = [torch.from_numpy(l_).to(DEV) for _, l_ in vids]
    assert blocks_mod._batchable(net, seqs)
    with torch.no_grad():
        saves = net(seqs, labs, compute_loss=False)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    P = {n: p.detach().double().cpu() for n, p in net.named_parameters()}
    for v, (feats, _) in enumerate(vids):
        with torch.no_grad():
            out = fo.forward(spec, P, torch.from_numpy(feats).double())
            pred = fo.predict(spec, out, text.double().cpu())
        np.testing.assert_array_equal(saves[v]["pred"], pred.numpy(), err_msg=f"video {v}")
        if v == len(vids) - 1:   # the attributes hold the last video, as in the reference
            for i, (blk, rec) in enumerate(zip(net.block_list, out["blocks"])):
                if rec["type"] == "U":
                    np.testing.assert_array_equal(blk.tdu.start32.cpu().numpy(), rec["tdu"].starts)
                    np.testing.assert_array_equal(blk.tdu.end32.cpu().numpy(), rec["tdu"].ends)
                err = (blk.frame_clogit[:, 0].double().cpu() - rec["frame_clogit"]).abs().max().item()
                assert err < 1e-3, f"block {i}: per-frame logits differ by {err}"


@pytest.mark.parametrize("name", ["tiny_clip", "tiny_clip_iid"])
def test_pos_sink_matches_autograd_adds(name, monkeypatch):
    """The action-query table's readers accumulating into one shared buffer (fxf.PosGradSink) give the
    same parameter gradients as autograd adding their returned position gradients (FX_POS_SINK=0),
    up to the summation order."""
    from factmx import functional as fxf
    fx = load_fixture(name)
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    feats, label, _ = tiny_inputs(meta)
    T, D = feats.shape
    f2, l2 = pg.segmented_video(T + 9, D, sorted(set(label.tolist())), 5, seed=12, noise=0.4)
    seqs = [torch.from_numpy(feats).float().to(DEV), torch.from_numpy(f2).float().to(DEV)]
    labs = [torch.from_numpy(label).to(DEV), torch.from_numpy(l2).to(DEV)]
    monkeypatch.setattr(fxf, "POS_SINK", 0)
    ref = _run(_model(meta, cfg), seqs, labs, True, monkeypatch)
    monkeypatch.setattr(fxf, "POS_SINK", 1)
    got = _run(_model(meta, cfg), seqs, labs, True, monkeypatch)
    assert got[0] == pytest.approx(ref[0], rel=1e-6)
    assert ref[3]["action_query"].abs().max().item() > 0
    for n, g in ref[3].items():
        err = (got[3][n] - g).abs().max().item()
        assert err <= 1e-5 * g.abs().max().item() + 1e-7, (n, err)
