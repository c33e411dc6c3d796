"""Pin the CPU oracle to golden vectors captured from the reference (CPU-only).

The fixtures were produced by tests/golden/make_golden.py, which imports the
reference in place (build container only) and runs it in float64.
"""
import numpy as np
import pytest
import torch

import paramgen as pg
from helpers import (load_fixture, tiny_meta, cfg_from_meta, tiny_inputs, param_dict, check_grad)
from oracle import fact_oracle as fo
from oracle import segments as seglib

# ---------------------------------------------------------------------------
# integer segmentation (bit-exact)
# ---------------------------------------------------------------------------


def test_segments_golden():
    fx = load_fixture("segments")
    cases = sorted({k.split("/")[0] for k in fx.files})
    assert cases
    for c in cases:
        lab = fx[f"{c}/label"]
        a, s, e = seglib.run_length_segments(lab)
        np.testing.assert_array_equal(s, fx[f"{c}/start"])
        np.testing.assert_array_equal(e, fx[f"{c}/end"])
        np.testing.assert_array_equal(a, fx[f"{c}/action"])
        tr, sid = seglib.transcript_and_segment_ids(lab)
        np.testing.assert_array_equal(tr, fx[f"{c}/transcript"])
        np.testing.assert_array_equal(sid, fx[f"{c}/seg_id"])


def test_segments_edge_cases():
    with pytest.raises(ValueError):
        seglib.run_length_segments(np.array([], dtype=np.int64))
    a, s, e = seglib.run_length_segments(np.array([5]))
    assert list(s) == [0] and list(e) == [0] and list(a) == [5]
    c = seglib.segment_centers(np.array([0, 3]), np.array([2, 8]))
    assert list(c) == [1, 5]


# ---------------------------------------------------------------------------
# tiny end-to-end models
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("name", ["tiny_clip", "tiny_clip_iid", "tiny_fact_m2"])
def test_oracle_end_to_end(name):
    fx = load_fixture(name)
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    clip = meta["model"] == "FACT_CLIP"
    spec = fo.resolve_spec(cfg, meta["D"], meta["C"], clip=clip)
    P = param_dict(meta["param_shapes"], meta["seed"])
    feats, label, text = tiny_inputs(meta)
    text_t = torch.from_numpy(text) if clip else None
    # fpos on: the reference's float32 sinusoid table (basic.py:92-103) depends on the host's float32
    # exp/sin/cos, so the fixture carries the reference's own table and the oracle takes it as given
    pe = torch.from_numpy(fx["frame_pe"]) if spec["fpos"] else None
    out = fo.forward(spec, P, torch.from_numpy(feats), pe_table=pe)
    pred = fo.predict(spec, out, text_t)
    total, fact, con, m = fo.video_loss(spec, out, label, text_t)
    total.backward()

    tol = dict(rtol=1e-9, atol=1e-11)
    ltol = 1e-10
    for i, rec in enumerate(out["blocks"]):
        p = f"block{i}/"
        np.testing.assert_allclose(rec["frame_clogit"].detach().numpy(), fx[p + "frame_clogit"], **tol)
        np.testing.assert_allclose(rec["action_clogit"].detach().numpy(), fx[p + "action_clogit"], **tol)
        if rec["type"] != "i":
            np.testing.assert_allclose(rec["a2f_attn"].detach().numpy(), fx[p + "a2f_attn"], **tol)
            np.testing.assert_allclose(rec["f2a_attn"].detach().numpy(), fx[p + "f2a_attn"], **tol)
            np.testing.assert_allclose(rec["a2f_logit"].detach().numpy(), fx[p + "a2f_attn_logit"], **tol)
            np.testing.assert_allclose(rec["f2a_logit"].detach().numpy(), fx[p + "f2a_attn_logit"], **tol)
        if rec["type"] == "U":
            np.testing.assert_array_equal(rec["tdu"].starts, fx[p + "seg_start"])
            np.testing.assert_array_equal(rec["tdu"].ends, fx[p + "seg_end"])
            np.testing.assert_allclose(rec["seg_clogit"].detach().numpy(), fx[p + "seg_clogit"], **tol)
    np.testing.assert_array_equal(pred.numpy(), fx["pred"])
    np.testing.assert_array_equal(m[0].numpy(), fx["match_a"])
    np.testing.assert_array_equal(m[1].numpy(), fx["match_s"])
    np.testing.assert_allclose(total.item(), fx["loss"][0], rtol=ltol)
    if clip:
        np.testing.assert_allclose(out["proj"].detach().numpy(), fx["proj"], **tol)
        np.testing.assert_allclose(fact.item(), fx["fact_loss"][0], rtol=ltol)
        np.testing.assert_allclose(con.item(), fx["contrastive_loss"][0], rtol=ltol)
    for n, t in P.items():
        check_grad(fx, "", n, t.grad, rtol=1e-7, atol=1e-10)


# ---------------------------------------------------------------------------
# per-layer vectors at benchmark widths
# ---------------------------------------------------------------------------

H, A, FF, NH, Q, T = 512, 256, 512, 8, 32, 256
SEED = 101


def _leaf(name, shape, scale=1.0):
    return torch.from_numpy(pg.randn(name, shape, SEED, scale)).requires_grad_(True)


def _params(shapes):
    return param_dict(shapes, SEED)


def _run_case(fx, prefix, outs, inputs, P, tol=2e-6):
    total = 0
    for k, o in enumerate(outs):
        ref = fx[f"{prefix}out{k}"]
        o_ = o.reshape(ref.shape)
        np.testing.assert_allclose(o_.detach().numpy(), ref, rtol=tol, atol=tol * 1e-2, err_msg=f"{prefix}out{k}")
        g = torch.from_numpy(pg.randn(f"{prefix}g{k}", ref.shape, SEED))
        total = total + (o_ * g).sum()
    total.backward()
    for k, (x, to_ref) in enumerate(inputs):
        check_grad(fx, prefix, f"in{k}", to_ref(x.grad), rtol=1e-5, atol=1e-7)
    for n, t in P.items():
        check_grad(fx, prefix, n.split("/", 1)[1] if "/" in n else n, t.grad, rtol=1e-5, atol=1e-7)


def _x2y_shapes(p):
    return {f"{p}X_K.weight": (H, H), f"{p}X_K.bias": (H,), f"{p}X_V.weight": (H, H), f"{p}X_V.bias": (H,),
            f"{p}Y_Q.weight": (H, H), f"{p}Y_Q.bias": (H,), f"{p}Y_W.weight": (A, 2 * H), f"{p}Y_W.bias": (A,)}


@pytest.mark.parametrize("direction", ["f2a", "a2f"])
def test_oracle_x2y(direction):
    fx = load_fixture("layers")
    pre = f"x2y_{direction}/"
    nx, ny = (T, Q) if direction == "f2a" else (Q, T)
    dxp, dyp = (H, A) if direction == "f2a" else (A, H)
    X, Y = _leaf(f"{direction}_X", (nx, 1, H)), _leaf(f"{direction}_Y", (ny, 1, H))
    Xp, Yp = _leaf(f"{direction}_Xp", (nx, 1, dxp), 0.5), _leaf(f"{direction}_Yp", (ny, 1, dyp), 0.5)
    P = {k: v for k, v in _params(_x2y_shapes("")).items()}
    out, logit, attn = fo.x2y(P, "", X[:, 0], Y[:, 0], Xp[:, 0], Yp[:, 0])
    sq = lambda g: g  # noqa: E731
    _run_case(fx, pre, (out, logit, attn), [(X, sq), (Y, sq), (Xp, sq), (Yp, sq)], P)


def _mha_shapes(p, kdim=None):
    if kdim is None:
        d = {f"{p}in_proj_weight": (3 * A, A)}
    else:
        d = {f"{p}q_proj_weight": (A, A), f"{p}k_proj_weight": (A, kdim), f"{p}v_proj_weight": (A, kdim)}
    d.update({f"{p}in_proj_bias": (3 * A,), f"{p}out_proj.weight": (A, A), f"{p}out_proj.bias": (A,)})
    return d


def _ffn_norm_shapes(n):
    d = {"linear1.weight": (FF, A), "linear1.bias": (FF,), "linear2.weight": (A, FF), "linear2.bias": (A,)}
    for i in range(1, n + 1):
        d[f"norm{i}.weight"] = (A,)
        d[f"norm{i}.bias"] = (A,)
    return d


def test_oracle_sca_layer():
    fx = load_fixture("layers")
    tgt, mem = _leaf("sca_tgt", (Q, 1, A)), _leaf("sca_mem", (T, 1, H))
    pos, qpos = _leaf("sca_pos", (T, 1, H), 0.5), _leaf("sca_qpos", (Q, 1, A), 0.5)
    shapes = dict(_mha_shapes("self_attn."), **_mha_shapes("multihead_attn.", kdim=H), **_ffn_norm_shapes(3))
    P = _params(shapes)
    y = fo.sca_layer(P, "", tgt[:, 0], mem[:, 0], pos[:, 0], qpos[:, 0], NH)
    sq = lambda g: g  # noqa: E731
    _run_case(fx, "sca/", (y,), [(tgt, sq), (mem, sq), (pos, sq), (qpos, sq)], P)


def test_oracle_sa_layer():
    fx = load_fixture("layers")
    tgt, pos = _leaf("sa_tgt", (Q, 1, A)), _leaf("sa_pos", (Q, 1, A), 0.5)
    P = _params(dict(_mha_shapes("multihead_attn."), **_ffn_norm_shapes(2)))
    y = fo.sa_layer(P, "", tgt[:, 0], pos[:, 0], NH)
    sq = lambda g: g  # noqa: E731
    _run_case(fx, "sa/", (y,), [(tgt, sq), (pos, sq)], P)


@pytest.mark.parametrize("tag,d,Tn,ln", [("drl_d1", 1, 256, False), ("drl_d64_ln", 64, 256, True),
                                         ("drl_d512", 512, 1100, False)])
def test_oracle_dilated_residual(tag, d, Tn, ln):
    fx = load_fixture("layers")
    x = _leaf(tag + "_x", (1, A, Tn))
    shapes = {"conv_dilated.weight": (A, A, 3), "conv_dilated.bias": (A,),
              "conv_1x1.weight": (A, A, 1), "conv_1x1.bias": (A,)}
    if ln:
        shapes.update({"norm.weight": (A,), "norm.bias": (A,)})
    P = _params(shapes)
    h = x[0].t()
    z = torch.relu(fo.dilated_conv3(h, P["conv_dilated.weight"], P["conv_dilated.bias"], d))
    y = h + fo.linear(z, P["conv_1x1.weight"], P["conv_1x1.bias"])
    if ln:
        y = fo.layer_norm(y, P["norm.weight"], P["norm.bias"])
    _run_case(fx, tag + "/", (y.t()[None],), [(x, lambda g: g)], P)


def test_oracle_mstcn_and_mstcn2():
    fx = load_fixture("layers")
    x = _leaf("mstcn_x", (120, 1, 64))
    sh = {"conv_1x1.weight": (32, 64, 1), "conv_1x1.bias": (32,), "conv_out.weight": (48, 32, 1),
          "conv_out.bias": (48,)}
    for i in range(4):
        sh.update({f"layers.{i}.conv_dilated.weight": (32, 32, 3), f"layers.{i}.conv_dilated.bias": (32,),
                   f"layers.{i}.conv_1x1.weight": (32, 32, 1), f"layers.{i}.conv_1x1.bias": (32,)})
    P = _params(sh)
    y = fo.mstcn(P, "", x[:, 0], 4, False, True)
    _run_case(fx, "mstcn/", (y,), [(x, lambda g: g)], P)

    x = _leaf("mstcn2_x", (120, 1, 64))
    sh = {"conv_1x1_in.weight": (32, 64, 1), "conv_1x1_in.bias": (32,), "conv_out.weight": (48, 32, 1),
          "conv_out.bias": (48,)}
    for i in range(4):
        for k in (1, 2):
            sh.update({f"conv_dilated_{k}.{i}.weight": (32, 32, 3), f"conv_dilated_{k}.{i}.bias": (32,)})
        sh.update({f"conv_fusion.{i}.weight": (32, 64, 1), f"conv_fusion.{i}.bias": (32,)})
    P = _params(sh)
    y = fo.mstcn2(P, "", x[:, 0], 4, True)
    _run_case(fx, "mstcn2/", (y,), [(x, lambda g: g)], P)


def test_oracle_gru():
    fx = load_fixture("layers")
    x = _leaf("gru_x", (40, 1, H))
    sh = {}
    for sfx in ("", "_reverse"):
        sh.update({f"weight_ih_l0{sfx}": (3 * A, H), f"weight_hh_l0{sfx}": (3 * A, A),
                   f"bias_ih_l0{sfx}": (3 * A,), f"bias_hh_l0{sfx}": (3 * A,)})
    P = _params(sh)
    y = fo.gru(P, "", x[:, 0], 1)
    _run_case(fx, "gru/", (y,), [(x, lambda g: g)], P)


def test_oracle_feature_projection():
    fx = load_fixture("layers")
    x = _leaf("proj_x", (128, 1, 437))
    P = _params({"projection.0.weight": (512, 437), "projection.0.bias": (512,), "projection.1.weight": (512,),
                 "projection.1.bias": (512,), "projection.4.weight": (512, 512), "projection.4.bias": (512,)})
    y = fo.feature_projection(P, "", x[:, 0])
    _run_case(fx, "proj/", (y,), [(x, lambda g: g)], P)


def test_oracle_losses():
    fx = load_fixture("layers")
    e = _leaf("nce_emb", (300, 1, 512))
    emb = e[:, 0] / e[:, 0].norm(dim=-1, keepdim=True).clamp_min(1e-12)
    emb.retain_grad()
    text = torch.from_numpy(pg.text_embeddings(70, seed=SEED))
    lo = fo.infonce(emb, text, torch.from_numpy(fx["infonce/labels"]), 0.1)
    lo.backward()
    np.testing.assert_allclose(lo.item(), fx["infonce/loss"][0], rtol=1e-10)
    np.testing.assert_allclose(emb.grad.numpy(), fx["infonce/demb"], rtol=1e-5, atol=1e-9)
    lg = _leaf("smooth_logit", (1, 300, 75), 3.0)
    sl = fo.smooth_loss(lg[0])
    sl.backward()
    np.testing.assert_allclose(sl.item(), fx["smooth/loss"][0], rtol=1e-10)
    np.testing.assert_allclose(lg.grad[0].numpy(), fx["smooth/dlogit"], rtol=1e-5, atol=1e-9)
