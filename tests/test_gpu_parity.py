"""End-to-end parity of the HIP FACT / FACT_CLIP path (GPU).

* tiny configs vs golden vectors captured from the reference (float64 run):
  per-frame logits within 1e-4 (north star: 1e-3), TDU segment boundaries,
  Hungarian match and predictions bit-exact, loss and every parameter
  gradient within fp32 tolerance.
* benchmark shape (T=4096, D=2048, Nact=32, C=75, HAViD dims) vs the CPU oracle
  on the same seeded inputs: logits within 1e-3, boundaries/preds identical.
"""
import numpy as np
import pytest
import torch

import paramgen as pg
from helpers import load_fixture, tiny_meta, cfg_from_meta, tiny_inputs, check_grad
from oracle import fact_oracle as fo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build_model(meta, cfg):
    from factmx.models.blocks import FACT, FACT_CLIP
    from factmx.models.loss import MatchCriterion
    C, D = meta["C"], meta["D"]
    _, _, text = tiny_inputs(meta)
    if meta["model"] == "FACT_CLIP":
        net = FACT_CLIP(cfg, D, C, text_embeddings=torch.from_numpy(text).float())
    else:
        net = FACT(cfg, D, C)
    shapes = {n: tuple(p.shape) for n, p in net.named_parameters()}
    assert shapes == {k: tuple(v) for k, v in meta["param_shapes"].items()}, "state_dict layout differs"
    with torch.no_grad():
        for n, p in net.named_parameters():
            p.copy_(torch.from_numpy(pg.param_value(n, p.shape, meta["seed"])))
    net.mcriterion = MatchCriterion(cfg, C, [])
    return net.to(DEV)


@pytest.mark.parametrize("name", ["tiny_clip", "tiny_clip_iid", "tiny_fact_m2"])
def test_tiny_end_to_end_vs_reference(name, monkeypatch):
    fx = load_fixture(name)
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    net = build_model(meta, cfg)
    net.train()
    feats, label, _ = tiny_inputs(meta)
    captured = {}
    orig = net.mcriterion.match

    def spy(*a, **k):
        r = orig(*a, **k)
        captured["m"] = r
        return r
    net.mcriterion.match = spy
    # lockstep path (every batch, single videos included): device match cost + host Hungarian
    from factmx.models import vloss as vl
    orig_em = vl.EarlyMatch.matches

    def spy_em(self, Q):
        r = orig_em(self, Q)
        captured["m"] = tuple(torch.from_numpy(x) for x in r[0])
        return r
    monkeypatch.setattr(vl.EarlyMatch, "matches", spy_em)
    seq = torch.from_numpy(feats).float().to(DEV)
    lab = torch.from_numpy(label).to(DEV)
    total, saves = net([seq], [lab], compute_loss=True)
    total.backward()
    torch.cuda.synchronize()

    for i, blk in enumerate(net.block_list):
        p = f"block{i}/"
        if hasattr(blk, "tdu"):
            np.testing.assert_array_equal(blk.tdu.start32.cpu().numpy(), fx[p + "seg_start"], err_msg=p)
            np.testing.assert_array_equal(blk.tdu.end32.cpu().numpy(), fx[p + "seg_end"], err_msg=p)
        np.testing.assert_allclose(blk.frame_clogit[:, 0].detach().cpu().numpy(), fx[p + "frame_clogit"],
                                   rtol=1e-4, atol=1e-4, err_msg=p + "frame_clogit")
        np.testing.assert_allclose(blk.action_clogit[:, 0].detach().cpu().numpy(), fx[p + "action_clogit"],
                                   rtol=1e-4, atol=1e-4, err_msg=p + "action_clogit")
        if hasattr(blk, "a2f_attn"):
            np.testing.assert_allclose(blk.a2f_attn[0].detach().cpu().numpy(), fx[p + "a2f_attn"], atol=1e-5)
            np.testing.assert_allclose(blk.f2a_attn_logit[0].detach().cpu().numpy(), fx[p + "f2a_attn_logit"],
                                       rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(saves[0]["pred"], fx["pred"])
    np.testing.assert_array_equal(captured["m"][0].numpy(), fx["match_a"])
    np.testing.assert_array_equal(captured["m"][1].numpy(), fx["match_s"])
    np.testing.assert_allclose(total.item(), fx["loss"][0], rtol=2e-5)
    if meta["model"] == "FACT_CLIP":
        np.testing.assert_allclose(net.projected_frame_embeddings[:, 0].detach().cpu().numpy(), fx["proj"],
                                   atol=2e-5)
    for n, prm in net.named_parameters():
        g = prm.grad
        assert g is not None, n
        rms = float(fx[f"gradsum/{n}"][1]) / np.sqrt(g.numel())
        # absolute floor: some gradients are analytically zero (e.g. key biases under a row softmax)
        check_grad(fx, "", n, g.cpu(), rtol=2e-3, atol=2e-3 * rms + 1e-6)


# ---------------------------------------------------------------------------
# benchmark shape vs the CPU oracle
# ---------------------------------------------------------------------------

def test_north_star_shape_vs_oracle():
    from bench import make_cfg, make_video, build_model as bench_model
    cfg = make_cfg()
    T, D, C = 4096, 2048, 75
    net, text = bench_model(cfg, D, C, device=DEV, seed=0)
    feats, label = make_video(T, D, C, cfg, seed=1)
    net.train()
    seq = torch.from_numpy(feats).to(DEV)
    lab = torch.from_numpy(label).to(DEV)
    with torch.no_grad():
        saves = net([seq], [lab], compute_loss=False)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    P = {n: p.detach().double().cpu() for n, p in net.named_parameters()}
    with torch.no_grad():
        out = fo.forward(spec, P, torch.from_numpy(feats).double())
        pred = fo.predict(spec, out, text.double().cpu())
    for i, (blk, rec) in enumerate(zip(net.block_list, out["blocks"])):
        if rec["type"] == "U":
            np.testing.assert_array_equal(blk.tdu.start32.cpu().numpy(), rec["tdu"].starts, err_msg=f"block {i}")
            np.testing.assert_array_equal(blk.tdu.end32.cpu().numpy(), rec["tdu"].ends, err_msg=f"block {i}")
        err = (blk.frame_clogit[:, 0].double().cpu() - rec["frame_clogit"]).abs().max().item()
        assert err < 1e-3, f"block {i}: per-frame logits differ by {err}"
    np.testing.assert_array_equal(saves[0]["pred"], pred.numpy())
