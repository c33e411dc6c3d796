"""Functional CPU restatement of FACT / FACT_CLIP (oracle; TEST INFRASTRUCTURE ONLY).

This is the checker for the HIP path: a plain PyTorch-CPU (fp32 or fp64)
restatement of the reference algorithm written as free functions over a
``state_dict``-shaped parameter dict (the reference is an ``nn.Module`` tree).
Backward comes from CPU autograd over these functions.

Every function cites the reference file:line (relative to /root/reference) it
restates.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.

Parity is pinned against golden vectors produced by the reference itself
(``tests/golden/make_golden.py``; checked in ``tests/test_oracle_golden.py``).
"""
import math

import numpy as np
import torch

from . import segments as seglib

# ---------------------------------------------------------------------------
# spec resolution (config -> per-block dims)
# ---------------------------------------------------------------------------

_BLOCK_KEYS = ("hid_dim", "dropout", "a", "a_nhead", "a_ffdim", "a_layers", "a_dim",
               "f", "f_layers", "f_ln", "f_dim", "f_ngp", "s_layers")


def _get(node, key, default=None):
    if isinstance(node, dict):
        return node.get(key, default)
    return getattr(node, key, default)


def resolve_spec(cfg, in_dim, n_classes, clip=True):
    """Per-block dims with the None-inheritance of ``update_from``
    (fact_clip/configs/utils.py:219-231) applied in block order exactly as
    ``FACT_CLIP.__init__`` does (blocks.py:591-604)."""
    base = {k: _get(cfg.Bi, k) for k in _BLOCK_KEYS}
    bi = dict(base)
    blocks = []
    for t in _get(cfg.FACT, "block"):
        if t == "i":
            b = dict(bi)
        elif t in "uU":
            node = cfg.Bu if t == "u" else cfg.BU
            b = {k: _get(node, k) for k in _BLOCK_KEYS}
            for k in b:
                if b[k] is None and base.get(k) is not None:
                    b[k] = base[k]
            base = b
        else:
            raise ValueError(t)
        b["type"] = t
        blocks.append(b)
    loss = {k: _get(cfg.Loss, k) for k in ("pc", "a2fc", "match", "bgw", "nullw", "sw")}
    spec = dict(D=in_dim, C=n_classes, Q=_get(cfg.FACT, "ntoken"), fpos=bool(_get(cfg.FACT, "fpos")),
                trans=bool(_get(cfg.FACT, "trans")), mwt=float(_get(cfg.FACT, "mwt")),
                blocks=blocks, loss=loss, clip=clip, bi_hid=bi["hid_dim"],
                holdout=list(_get(cfg, "holdout_classes", []) or []))
    if clip:
        spec["temp"] = float(_get(cfg.CLIP, "temp"))
        spec["fact_w"] = float(_get(cfg.CLIP, "fact_loss_weight"))
        spec["cont_w"] = float(_get(cfg.CLIP, "contrastive_weight"))
    if spec["trans"]:
        raise NotImplementedError("FACT.trans=True is not on the FACT_CLIP hot path")
    return spec


# ---------------------------------------------------------------------------
# layer primitives.  Layout: (rows, channels); the reference's (N, B=1, C)
# with the unit batch axis dropped.
# ---------------------------------------------------------------------------

def linear(x, w, b):
    """nn.Linear / Conv1d(k=1) on channel-last rows: x @ w^T + b."""
    if w.dim() == 3:          # Conv1d weight (out, in, 1)
        w = w[:, :, 0]
    y = x @ w.t()
    return y if b is None else y + b


def dilated_conv3(x, w, b, d):
    """Conv1d(k=3, dilation=d, padding=d) on (T, C) rows (basic.py:138): sum of three
    row-shifted GEMMs over a zero-padded copy."""
    T = x.shape[0]
    xp = torch.nn.functional.pad(x, (0, 0, d, d))
    y = b.clone().expand(T, -1) if b is not None else 0
    for j in range(3):
        y = y + xp[j * d: j * d + T] @ w[:, :, j].t()
    return y


def layer_norm(x, w, b, eps=1e-5):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def softmax(x, dim=-1):
    m = x.max(dim=dim, keepdim=True).values
    e = torch.exp(x - m)
    return e / e.sum(dim=dim, keepdim=True)


def log_softmax(x, dim=-1):
    m = x.max(dim=dim, keepdim=True).values
    z = x - m
    return z - torch.log(torch.exp(z).sum(dim=dim, keepdim=True))


def add_pos(x, pos):
    """``add_positional_encoding`` (basic.py:313-320): pos added to the first d channels."""
    if pos is None:
        return x
    d = pos.shape[-1]
    if d == x.shape[-1]:
        return x + pos
    return torch.cat([x[:, :d] + pos, x[:, d:]], dim=-1)


def sinusoid_table(n, d, empty):
    """``PositionalEncoding`` (basic.py:92-103, 114-129): computed in float32 as the reference does."""
    pe = torch.zeros(n, d, dtype=torch.float32)
    if not empty:
        pos = torch.arange(0, n, dtype=torch.float32).unsqueeze(1)
        div = torch.exp(torch.arange(0, d, 2).float() * (-math.log(10000.0) / d))
        pe[:, 0::2] = torch.sin(pos * div)
        pe[:, 1::2] = torch.cos(pos * div)
    return pe


def process_feature(x, n):
    """``Block.process_feature`` (blocks.py:195-202): last n channels -> softmax probs."""
    clogit = x[:, -n:]
    return torch.cat([x[:, :-n], softmax(clogit)], dim=-1), clogit


# ---------------------------------------------------------------------------
# modules
# ---------------------------------------------------------------------------

def mstcn(P, p, x, nlayers, ln, in_map):
    """``MSTCN.forward`` + ``DilatedResidualLayer.forward`` (basic.py:200-220, 154-171), eval-mode dropout."""
    h = linear(x, P[p + "conv_1x1.weight"], P[p + "conv_1x1.bias"]) if in_map else x
    for i in range(nlayers):
        q = f"{p}layers.{i}."
        z = torch.relu(dilated_conv3(h, P[q + "conv_dilated.weight"], P[q + "conv_dilated.bias"], 2 ** i))
        h = h + linear(z, P[q + "conv_1x1.weight"], P[q + "conv_1x1.bias"])
        if ln:
            h = layer_norm(h, P[q + "norm.weight"], P[q + "norm.bias"])
    return linear(h, P[p + "conv_out.weight"], P[p + "conv_out.bias"])


def mstcn2(P, p, x, nlayers, in_map):
    """``MSTCN2.forward`` (basic.py:263-281): dual dilation 2^(L-1-i) / 2^i, 1x1 fusion, ReLU, residual."""
    f = linear(x, P[p + "conv_1x1_in.weight"], P[p + "conv_1x1_in.bias"]) if in_map else x
    for i in range(nlayers):
        a = dilated_conv3(f, P[f"{p}conv_dilated_1.{i}.weight"], P[f"{p}conv_dilated_1.{i}.bias"], 2 ** (nlayers - 1 - i))
        b = dilated_conv3(f, P[f"{p}conv_dilated_2.{i}.weight"], P[f"{p}conv_dilated_2.{i}.bias"], 2 ** i)
        g = torch.relu(linear(torch.cat([a, b], -1), P[f"{p}conv_fusion.{i}.weight"], P[f"{p}conv_fusion.{i}.bias"]))
        f = g + f
    return linear(f, P[p + "conv_out.weight"], P[p + "conv_out.bias"])


def frame_branch(P, p, x, b, in_map):
    if b["f"] == "m":
        return mstcn(P, p, x, b["f_layers"], b["f_ln"], in_map)
    if b["f"] == "m2":
        return mstcn2(P, p, x, b["f_layers"], in_map)
    raise ValueError(b["f"])


def mha(P, p, q_in, k_in, v_in, nhead):
    """``nn.MultiheadAttention`` forward math as called in basic.py:442,500,513 (no dropout):
    per-head softmax(q k^T / sqrt(hd)) v, then out_proj."""
    E = q_in.shape[-1]
    hd = E // nhead
    bi = P[p + "in_proj_bias"]
    if (p + "in_proj_weight") in P:
        W = P[p + "in_proj_weight"]
        wq, wk, wv = W[:E], W[E:2 * E], W[2 * E:]
    else:
        wq, wk, wv = P[p + "q_proj_weight"], P[p + "k_proj_weight"], P[p + "v_proj_weight"]
    q = linear(q_in, wq, bi[:E])
    k = linear(k_in, wk, bi[E:2 * E])
    v = linear(v_in, wv, bi[2 * E:])
    L, S = q.shape[0], k.shape[0]
    qh = q.reshape(L, nhead, hd).transpose(0, 1)
    kh = k.reshape(S, nhead, hd).transpose(0, 1)
    vh = v.reshape(S, nhead, hd).transpose(0, 1)
    att = softmax(qh @ kh.transpose(1, 2) / math.sqrt(hd))
    o = (att @ vh).transpose(0, 1).reshape(L, E)
    return linear(o, P[p + "out_proj.weight"], P[p + "out_proj.bias"])


def sca_layer(P, p, tgt, mem, pos, qpos, nhead):
    """``SCALayer.forward`` (basic.py:494-523), post-norm, eval dropout."""
    q = add_pos(tgt, qpos)
    tgt = layer_norm(tgt + mha(P, p + "self_attn.", q, q, tgt, nhead), P[p + "norm1.weight"], P[p + "norm1.bias"])
    q = add_pos(tgt, qpos)
    k = add_pos(mem, pos)
    tgt = layer_norm(tgt + mha(P, p + "multihead_attn.", q, k, mem, nhead), P[p + "norm2.weight"], P[p + "norm2.bias"])
    ff = linear(torch.relu(linear(tgt, P[p + "linear1.weight"], P[p + "linear1.bias"])),
                P[p + "linear2.weight"], P[p + "linear2.bias"])
    return layer_norm(tgt + ff, P[p + "norm3.weight"], P[p + "norm3.bias"])


def sca_decoder(P, p, tgt, mem, pos, qpos, nlayers, nhead):
    """``SCADecoder.forward`` (basic.py:542-557) with the final LayerNorm of create_abranch (blocks.py:223)."""
    for i in range(nlayers):
        tgt = sca_layer(P, f"{p}layers.{i}.", tgt, mem, pos, qpos, nhead)
    tgt = layer_norm(tgt, P[p + "norm.weight"], P[p + "norm.bias"])
    return linear(tgt, P[p + "out_linear.weight"], P[p + "out_linear.bias"])


def sa_layer(P, p, tgt, pos, nhead):
    """``SALayer.forward`` (basic.py:429-452) as called by SADecoder (q=k=tgt+pos, v=tgt)."""
    q = add_pos(tgt, pos)
    tgt = layer_norm(tgt + mha(P, p + "multihead_attn.", q, q, tgt, nhead), P[p + "norm1.weight"], P[p + "norm1.bias"])
    ff = linear(torch.relu(linear(tgt, P[p + "linear1.weight"], P[p + "linear1.bias"])),
                P[p + "linear2.weight"], P[p + "linear2.bias"])
    return layer_norm(tgt + ff, P[p + "norm2.weight"], P[p + "norm2.bias"])


def sa_decoder(P, p, tgt, pos, nlayers, nhead):
    """``SADecoder.forward`` (basic.py:578-593)."""
    for i in range(nlayers):
        tgt = sa_layer(P, f"{p}layers.{i}.", tgt, pos, nhead)
    return linear(tgt, P[p + "out_linear.weight"], P[p + "out_linear.bias"])


def x2y(P, p, X, Y, Xpos, Ypos):
    """``X2Y_map.forward`` (basic.py:349-389), kq_pos=True (blocks.py:234-240).
    Returns (Y_out, logit (Y, X), attn (Y, X))."""
    xk = linear(add_pos(X, Xpos), P[p + "X_K.weight"], P[p + "X_K.bias"])
    xv = linear(X, P[p + "X_V.weight"], P[p + "X_V.bias"])
    yq = linear(add_pos(Y, Ypos), P[p + "Y_Q.weight"], P[p + "Y_Q.bias"])
    logit = yq @ xk.t() / math.sqrt(xk.shape[-1])
    attn = softmax(logit, -1)
    out = linear(torch.cat([Y, attn @ xv], -1), P[p + "Y_W.weight"], P[p + "Y_W.bias"])
    return out, logit, attn


def gru(P, p, x, nlayers):
    """Bidirectional ``nn.GRU`` (blocks.py:401,432) restated: gates (r, z, n), h0 = 0,
    output = concat(forward, backward) per step."""
    inp = x
    for layer in range(nlayers):
        outs = []
        for sfx, reverse in (("", False), ("_reverse", True)):
            wih = P[f"{p}weight_ih_l{layer}{sfx}"]
            whh = P[f"{p}weight_hh_l{layer}{sfx}"]
            bih = P[f"{p}bias_ih_l{layer}{sfx}"]
            bhh = P[f"{p}bias_hh_l{layer}{sfx}"]
            Hh = whh.shape[1]
            gi = inp @ wih.t() + bih
            h = torch.zeros(Hh, dtype=x.dtype)
            res = [None] * inp.shape[0]
            order = range(inp.shape[0] - 1, -1, -1) if reverse else range(inp.shape[0])
            for t in order:
                gh = h @ whh.t() + bhh
                r = torch.sigmoid(gi[t, :Hh] + gh[:Hh])
                z = torch.sigmoid(gi[t, Hh:2 * Hh] + gh[Hh:2 * Hh])
                n = torch.tanh(gi[t, 2 * Hh:] + r * gh[2 * Hh:])
                h = (1 - z) * n + z * h
                res[t] = h
            outs.append(torch.stack(res, 0))
        inp = torch.cat(outs, -1)
    return inp


def feature_projection(P, p, x):
    """``FeatureProjection.forward`` (blocks.py:153-175): Linear, LN, ReLU, Linear, L2-normalise."""
    h = linear(x, P[p + "projection.0.weight"], P[p + "projection.0.bias"])
    h = torch.relu(layer_norm(h, P[p + "projection.1.weight"], P[p + "projection.1.bias"]))
    h = linear(h, P[p + "projection.4.weight"], P[p + "projection.4.bias"])
    nrm = torch.sqrt((h * h).sum(-1, keepdim=True)).clamp_min(1e-12)
    return h / nrm


# ---------------------------------------------------------------------------
# whole model forward
# ---------------------------------------------------------------------------

class TDU:
    """Integer state of ``TemporalDownsampleUpsample`` (basic.py:595-651)."""

    def __init__(self, pred):
        self.action, self.starts, self.ends = seglib.run_length_segments(pred)
        self.num_seg = len(self.starts)
        n = len(pred)
        self.seg_label = torch.from_numpy(seglib.segment_ids_from_bounds(self.starts, self.ends, n))
        self.seg_lens = torch.from_numpy(self.ends - self.starts + 1)
        self.centers = torch.from_numpy(seglib.segment_centers(self.starts, self.ends))

    def frame2seg(self, f):
        out = torch.zeros(self.num_seg, f.shape[1], dtype=f.dtype).index_add(0, self.seg_label, f)
        return out / self.seg_lens[:, None].to(f.dtype)


def forward(spec, P, seq, pe_table=None):
    """``FACT_CLIP._forward_one_video`` (blocks.py:610-675) for one video, eval-mode dropout,
    no channel masking / time mask.  Returns a dict with every side-channel tensor
    the losses and eval read."""
    C, Q = spec["C"], spec["Q"]
    T = seq.shape[0]
    dt = seq.dtype
    H0 = spec["blocks"][0]["hid_dim"]
    if pe_table is None:
        pe_table = sinusoid_table(T, H0, empty=not spec["fpos"])
    frame_pos = pe_table[:T].to(dt)
    action_pos = P["action_query"][:, 0, :]
    action = torch.zeros_like(action_pos)
    frame = seq
    out = {"blocks": []}
    for bi, b in enumerate(spec["blocks"]):
        p = f"block_list.{bi}."
        rec = {"type": b["type"]}
        nh = b["a_nhead"]
        if b["type"] == "i":                                     # InputBlock.forward blocks.py:295-311
            frame = frame_branch(P, p + "frame_branch.", frame, b, in_map=True)
            frame, rec["frame_clogit"] = process_feature(frame, C)
            action = sca_decoder(P, p + "action_branch.", action, frame, frame_pos, action_pos, b["a_layers"], nh)
            action, rec["action_clogit"] = process_feature(action, C + 1)
        elif b["type"] == "u":                                   # UpdateBlock.forward blocks.py:343-367
            action, rec["f2a_logit"], rec["f2a_attn"] = x2y(P, p + "f2a_layer.", frame, action, frame_pos, action_pos)
            action = sa_decoder(P, p + "action_branch.", action, action_pos, b["a_layers"], nh)
            action, rec["action_clogit"] = process_feature(action, C + 1)
            frame, rec["a2f_logit"], rec["a2f_attn"] = x2y(P, p + "a2f_layer.", action, frame, action_pos, frame_pos)
            frame = frame_branch(P, p + "frame_branch.", frame, b, in_map=False)
            frame, rec["frame_clogit"] = process_feature(frame, C)
        else:                                                    # UpdateBlockTDU.forward blocks.py:449-485
            pred = frame[:, -C:].detach().max(dim=-1).indices.numpy()
            tdu = TDU(pred)
            seg = tdu.frame2seg(frame)
            seg = torch.relu(gru(P, p + "seg_update.", seg, b["s_layers"]))
            seg = linear(seg, P[p + "seg_combine.weight"], P[p + "seg_combine.bias"])
            seg, rec["seg_clogit"] = process_feature(seg, C)
            seg_pos = frame_pos[tdu.centers]
            action, f2a_logit, f2a_attn = x2y(P, p + "f2a_layer.", seg, action, seg_pos, action_pos)
            action = sa_decoder(P, p + "action_branch.", action, action_pos, b["a_layers"], nh)
            action, rec["action_clogit"] = process_feature(action, C + 1)
            seg, a2f_logit, a2f_attn = x2y(P, p + "a2f_layer.", action, seg, action_pos, seg_pos)
            s2f = seg[tdu.seg_label]
            frame = torch.relu(linear(torch.cat([s2f, frame], -1), P[p + "sf_merge.0.weight"], P[p + "sf_merge.0.bias"]))
            frame = frame_branch(P, p + "frame_branch.", frame, b, in_map=False)
            frame, rec["frame_clogit"] = process_feature(frame, C)
            rec.update(tdu=tdu, f2a_logit=f2a_logit, a2f_logit=a2f_logit,
                       f2a_attn=f2a_attn[:, tdu.seg_label], a2f_attn=a2f_attn[tdu.seg_label])
        rec["frame_feature"] = frame
        rec["action_feature"] = action
        out["blocks"].append(rec)
    if spec["clip"]:
        feat_dim = frame.shape[-1] - C
        out["proj"] = feature_projection(P, "frame_projection.", frame[:, :feat_dim])
    return out


# ---------------------------------------------------------------------------
# eval decode
# ---------------------------------------------------------------------------

def _abranch(last):
    """Shared part of ``Block._eval`` (blocks.py:243-261) / ``eval_with_clip`` (blocks.py:854-869)."""
    acl = last["action_clogit"]
    a2f = last["a2f_attn"]
    tok_pred = acl.argmax(1)
    null = acl.shape[-1] - 1
    loc = torch.nonzero(tok_pred != null)[:, 0]
    if len(loc) == 0:
        return None
    qtk = softmax(acl[:, :-1], 1)
    which = loc[a2f[:, loc].argmax(-1)]
    return qtk[which]


def predict(spec, out, text_emb=None):
    """Per-frame prediction: ``eval_with_clip`` (blocks.py:788-887) for FACT_CLIP with text
    embeddings, else ``Block._eval`` (blocks.py:243-261)."""
    last = out["blocks"][-1]
    mwt = spec["mwt"]
    if spec["clip"] and text_emb is not None:
        clip_prob = softmax(out["proj"] @ text_emb.t() / spec["temp"], -1)
        ab = _abranch(last)
        if ab is None:
            return clip_prob.argmax(1)
        return ((1 - mwt) * ab + mwt * clip_prob).argmax(1)
    fprob = softmax(last["frame_clogit"], -1)
    ab = _abranch(last)
    if ab is None:
        return fprob.argmax(1)
    return ((1 - mwt) * ab + mwt * fprob).argmax(1)


# ---------------------------------------------------------------------------
# matching + losses (fact_clip/models/loss.py)
# ---------------------------------------------------------------------------

class LabelState:
    """``MatchCriterion.set_label`` (loss.py:58-84)."""

    def __init__(self, spec, label, bg_ids=(), dtype=torch.float64):
        C = spec["C"]
        lab = np.asarray(label, dtype=np.int64)
        tr, sid = seglib.transcript_and_segment_ids(lab)
        self.class_label = torch.from_numpy(lab)
        self.transcript = torch.from_numpy(tr)
        self.seg_label = torch.from_numpy(sid)
        T = len(lab)
        self.onehot_class = torch.zeros(T, C, dtype=dtype)
        self.onehot_class[torch.arange(T), self.class_label] = 1
        self.onehot_seg = torch.zeros(T, len(tr), dtype=dtype)
        self.onehot_seg[torch.arange(T), self.seg_label] = 1
        cw = torch.ones(C + 1, dtype=dtype)
        cw[-1] = spec["loss"]["nullw"]
        for i in bg_ids:
            cw[i] = spec["loss"]["bgw"]
        sw = torch.ones(len(tr), dtype=dtype)
        for i in bg_ids:
            sw[self.transcript == i] = spec["loss"]["bgw"]
        self.cweight, self.sweight = cw, sw


def soft_iou(a2f_attn, onehot_seg):
    """``MatchCriterion.a2f_soft_iou`` (loss.py:91-106) in numpy."""
    a = a2f_attn.detach().numpy()[:, :, None]            # t, a, 1
    s = onehot_seg.numpy()[:, None, :]                   # t, 1, s
    overlap = np.einsum('tax,txs->as', a, s)
    union = np.minimum(a + s, 1.0).sum(0)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.nan_to_num(overlap / union, nan=0.0)


def match(spec, ls, action_clogit, a2f_attn):
    """``MatchCriterion.match`` (loss.py:108-153); o2o via scipy Hungarian."""
    from scipy.optimize import linear_sum_assignment
    cfg = spec["loss"]
    S = ls.onehot_seg.shape[1]
    if cfg["match"] == "seq":
        idx = torch.arange(S)
        return idx, idx
    cost = 0
    if cfg["pc"] > 0:
        prob = softmax(action_clogit.detach(), -1)[:, ls.transcript].numpy()
        cost = cost - cfg["pc"] * prob
    if cfg["a2fc"] > 0:
        cost = cost - cfg["a2fc"] * soft_iou(a2f_attn, ls.onehot_seg)
    cost = np.asarray(cost)
    if cfg["match"] == "o2o":
        ai, si = linear_sum_assignment(cost)
    elif cfg["match"] == "o2m":
        ai, si = _one_to_many(ls, cost)
    else:
        raise ValueError(cfg["match"])
    return torch.as_tensor(np.asarray(ai), dtype=torch.int64), torch.as_tensor(np.asarray(si), dtype=torch.int64)


def _one_to_many(ls, cost):
    """``MatchCriterion._one_to_many_match`` (loss.py:155-193)."""
    from scipy.optimize import linear_sum_assignment
    tr = ls.transcript.numpy()
    actions = np.unique(tr)
    t2a = np.stack([cost[:, tr == a].sum(1) for a in actions], 1)
    aid, cid = linear_sum_assignment(t2a)
    un_a = [a for a in range(cost.shape[0]) if a not in aid]
    un_c = t2a[un_a].argmin(1)
    all_a = np.array(aid.tolist() + un_a)
    all_c = np.array([actions[i] for i in cid.tolist() + un_c.tolist()])
    tok_cls = np.zeros(cost.shape[0])
    tok_cls[all_a] = all_c
    m = {}
    for a in actions:
        sw = np.where(tr == a)[0]
        tw = np.where(tok_cls == a)[0]
        asg = cost[tw][:, sw].argmin(0)
        for s, k in zip(sw, asg):
            m[s] = tw[k]
    return list(m.values()), list(m.keys())


def smooth_loss(logit):
    """``smooth_loss`` (loss.py:8-18) on (T, C)."""
    ls = log_softmax(logit, -1)
    return torch.clamp((ls[1:] - ls[:-1]) ** 2, min=0, max=16).mean()


def frame_loss(ls, clogit):
    """``frame_loss`` (loss.py:246-258)."""
    C = clogit.shape[-1]
    lp = log_softmax(clogit, -1)
    return (-lp * ls.onehot_class * ls.cweight[:C]).sum() / ls.onehot_class.sum()


def zoom(tdu, onehot):
    z = torch.zeros(tdu.num_seg, onehot.shape[1], dtype=onehot.dtype).index_add(0, tdu.seg_label, onehot)
    return z / tdu.seg_lens[:, None].to(onehot.dtype)


def frame_loss_tdu(ls, seg_clogit, tdu):
    """``frame_loss_tdu`` (loss.py:260-277)."""
    lp = log_softmax(seg_clogit, -1)
    z = zoom(tdu, ls.onehot_class)
    return (-lp * z * ls.cweight[:lp.shape[-1]]).sum() / z.sum()


def token_loss(ls, m, action_clogit):
    """``action_token_loss`` (loss.py:195-207): weighted CE, null class default."""
    ai, si = m
    A, Cp = action_clogit.shape
    tgt = torch.full((A,), Cp - 1, dtype=torch.int64)
    tgt[ai] = ls.transcript[si]
    lp = log_softmax(action_clogit, -1)
    w = ls.cweight[tgt]
    return (-(lp[torch.arange(A), tgt]) * w).sum() / w.sum()


def cross_attn_loss(ls, m, attn, axis, tdu=None):
    """``cross_attn_loss`` / ``cross_attn_loss_tdu`` (loss.py:209-244).  ``attn`` is (rows, tokens);
    axis 0 = log-softmax over rows (the f2a call, dim=1), axis 1 = over matched tokens (a2f, dim=2).
    sweight multiplies matched column i by sweight[i] exactly as the reference broadcasts."""
    ai, si = m
    tgt_full = ls.onehot_seg if tdu is None else zoom(tdu, ls.onehot_seg)
    tgt = tgt_full[:, si]
    a = attn[:, ai]
    lp = log_softmax(a, axis)
    l2 = -lp * tgt * ls.sweight
    return l2.sum() / tgt_full.sum()


def block_loss(spec, ls, rec, m):
    """``compute_loss`` of the three block kinds (blocks.py:313-320, 369-382, 487-497)."""
    sw = spec["loss"]["sw"]
    fl = frame_loss(ls, rec["frame_clogit"])
    atk = token_loss(ls, m, rec["action_clogit"])
    sm = smooth_loss(rec["frame_clogit"])
    if rec["type"] == "i":
        return fl + atk + sw * sm
    if rec["type"] == "u":
        f2a = cross_attn_loss(ls, m, rec["f2a_logit"].t(), 0)
        a2f = cross_attn_loss(ls, m, rec["a2f_logit"], 1)
        sm = smooth_loss(rec["a2f_logit"]) + smooth_loss(rec["f2a_logit"].t()) + sm
        return atk + f2a + a2f + fl + sw * sm
    tdu = rec["tdu"]
    sl = frame_loss_tdu(ls, rec["seg_clogit"], tdu)
    f2a = cross_attn_loss(ls, m, rec["f2a_logit"].t(), 0, tdu)
    a2f = cross_attn_loss(ls, m, rec["a2f_logit"], 1, tdu)
    return (fl + sl) / 2 + atk + f2a + a2f + sw * sm


def infonce(emb, text, labels, temp):
    """``infonce_contrastive_loss`` (loss.py:280-341) with B=1."""
    sim = emb @ text.t() / temp
    n = text.shape[0]
    lp = log_softmax(sim, -1)
    v2t = -lp[torch.arange(len(labels)), labels].mean()
    tgt = torch.zeros(len(labels), n, dtype=emb.dtype)
    tgt[torch.arange(len(labels)), labels] = 1
    lpt = log_softmax(sim.t(), 1)
    cnt = tgt.sum(0).clamp(min=1.0)
    t2v = (-(lpt * tgt.t()).sum(1) / cnt).mean()
    return (v2t + t2v) / 2


def video_loss(spec, out, label, text_emb=None, bg_ids=()):
    """``FACT_CLIP._loss_one_video`` (blocks.py:677-786) / ``FACT._loss_one_video`` (blocks.py:90-106).
    Returns (total, fact_loss, contrastive_loss or None, match)."""
    dt = out["blocks"][-1]["frame_feature"].dtype
    ls = LabelState(spec, label, bg_ids, dtype=dt)
    last = out["blocks"][-1]
    m = match(spec, ls, last["action_clogit"], last["a2f_attn"])
    losses = [block_loss(spec, ls, rec, m) for rec in out["blocks"]]
    fact = sum(losses) / len(losses)
    if not spec["clip"] or text_emb is None:
        return fact, fact, None, m
    emb = out["proj"]
    text = text_emb
    lab = ls.class_label
    if spec["holdout"]:
        n = text_emb.shape[0]
        hold = set(spec["holdout"])
        seen = torch.tensor([i for i in range(n) if i not in hold], dtype=torch.int64)
        text = text_emb[seen]
        mapper = torch.full((n,), -1, dtype=torch.int64)
        mapper[seen] = torch.arange(len(seen))
        lab = mapper[lab]
        if (lab == -1).any():
            keep = lab != -1
            if keep.sum() == 0:
                return fact, fact, None, m
            lab = lab[keep]
            emb = emb[keep]
    con = infonce(emb, text, lab, spec["temp"])
    total = spec["fact_w"] * fact + spec["cont_w"] * con
    return total, fact, con, m
