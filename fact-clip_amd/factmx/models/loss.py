"""Matching and losses with the reference's surface (fact_clip/models/loss.py).

Label bookkeeping is vectorised on the label's device (the reference loops over
frames in Python).  The Hungarian assignment stays on the host (scipy, as in
the reference); its cost matrix (tokens x GT segments) is built on the device
and copied once.  The per-term losses run as fused HIP kernel pairs
(functional.ClassLossFn / AttnLossFn); a lockstep batch of videos takes the
whole loss phase through models/vloss.py instead (a handful of launches for
every term of every video).
"""
import numpy as np
import torch
import torch.nn.functional as F
from scipy.optimize import linear_sum_assignment

from .. import functional as fxf
from . import basic
from .basic import torch_class_label_to_segment_label, logit2prob  # noqa: F401  (re-exported like loss.py:20,38)


def smooth_loss(logit, is_logit=True):
    """loss.py:8-18: mean of clamp((d/dt log_softmax)^2, 0, 16) over (B, T-1, C)."""
    lp = F.log_softmax(logit, dim=2) if is_logit else logit
    step = lp[:, 1:] - lp[:, :-1]
    return torch.clamp(step * step, min=0, max=16).mean()


def _to_dev(t, dev):
    """Host -> device without a device drain: a non-blocking copy through torch's caching pinned
    allocator (the staging block is reused once its copy has completed, no per-call pinning)."""
    if t.device == dev or dev.type == "cpu":
        return t.to(dev)
    staged = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    staged.copy_(t)
    return staged.to(dev, non_blocking=True)


def _onehot(idx, n):
    return F.one_hot(idx.to(torch.int64), n).to(torch.float32)


def _zoom(tdu, onehot):
    """Mean of a frame-level (T, K) table over each TDU segment -> (S, K)."""
    z = torch.zeros(tdu.num_seg, onehot.shape[1], dtype=onehot.dtype, device=onehot.device)
    z.index_add_(0, tdu.seg_label, onehot)
    return z / tdu.seg_lens[:, None]


def _weighted_xent(logits, target, weight):
    """Mean cross-entropy with class weights: sum w[y] * nll / sum w[y] (F.cross_entropy semantics)."""
    return F.cross_entropy(logits, target, weight=weight)


class MatchCriterion:
    """loss.py:49-277."""

    def __init__(self, cfg, nclasses, bg_ids=[], class_weight=None):
        self.cfg = cfg
        self.nclasses = nclasses
        self.bg_ids = list(bg_ids) if bg_ids is not None else []
        self._class_weight = class_weight

    def set_label(self, label, label_host=None):
        """loss.py:58-84.  ``label_host`` = (cpu tensor, cuda event) from an asynchronous copy
        started earlier (FACT*.forward): the run-length transcript is then built on the host
        without draining the device; without it the device path below is used."""
        self.class_label = label
        dev = label.device
        lab_np = None
        if label_host is not None:
            lh, ev = label_host
            if ev is not None:
                ev.synchronize()
            lab_np = lh.numpy()
        elif not label.is_cuda:
            lab_np = label.numpy()
        self._label_np = lab_np
        if lab_np is not None:
            change = np.ones(len(lab_np), dtype=bool)
            change[1:] = lab_np[1:] != lab_np[:-1]
            self._transcript_np = lab_np[change].astype(np.int64)
            self.transcript = _to_dev(torch.from_numpy(self._transcript_np), dev)
            self.seg_label = _to_dev(torch.from_numpy((np.cumsum(change) - 1).astype(lab_np.dtype)), dev)
        else:
            self.transcript, self.seg_label = torch_class_label_to_segment_label(label)
            self._transcript_np = None
        S = int(self.transcript.shape[0])
        self._sweight_np = None
        if self._transcript_np is not None:
            if self._class_weight is not None:
                self._sweight_np = np.asarray(self._class_weight, dtype=np.float32)[self._transcript_np]
            else:
                swn = np.ones(S, dtype=np.float32)
                for i in self.bg_ids:
                    swn[self._transcript_np == i] = self.cfg.Loss.bgw
                self._sweight_np = swn
        self.onehot_class_label = _onehot(label, self.nclasses)
        self.onehot_seg_label = _onehot(self.seg_label, S)
        cw = torch.ones(self.nclasses + 1, device=dev)
        cw[-1] = self.cfg.Loss.nullw
        sw = torch.ones(S, dtype=torch.float32, device=dev)
        if self._class_weight is not None:
            cw[:self.nclasses] = torch.as_tensor(self._class_weight[:self.nclasses], dtype=torch.float32, device=dev)
            sw = torch.as_tensor(self._class_weight, dtype=torch.float32, device=dev)[self.transcript]
        else:
            for i in self.bg_ids:
                cw[i] = self.cfg.Loss.bgw
                sw = torch.where(self.transcript == i, torch.full_like(sw, self.cfg.Loss.bgw), sw)
        self.cweight, self.sweight = cw, sw
        self._match_cache = None

    def _label_to_onehot(self, label, nclass):
        return _onehot(label, nclass)

    @classmethod
    def a2f_soft_iou(cls, a2f_attn, onehot_seg_label):
        """loss.py:91-106 on the device: overlap / sum_t min(attn + onehot, 1)."""
        a = a2f_attn[0]                                      # (T, A)
        if a.is_cuda:
            overlap = fxf.matmul_tn(a, onehot_seg_label)     # (A, S), one fx_gemm
        else:
            overlap = a.t() @ onehot_seg_label
        union = torch.minimum(a[:, :, None] + onehot_seg_label[:, None, :], torch.ones((), device=a.device)).sum(0)
        return torch.nan_to_num(overlap / union, nan=0.0)

    def match(self, clogit, a2f_attn):
        """loss.py:108-153: Hungarian (o2o) / one-to-many / sequential matching."""
        assert clogit.shape[1] == 1
        mcfg = self.cfg.Loss
        S = self.onehot_seg_label.shape[-1]
        if mcfg.match == "seq":
            A = clogit.shape[0]
            assert A >= S, (A, S)
            idx = torch.arange(S, dtype=torch.int64)
            return idx, idx
        with torch.no_grad():
            cost = torch.zeros(clogit.shape[0], S, device=clogit.device)
            if mcfg.pc > 0:
                cost = cost - mcfg.pc * clogit.squeeze(1)[:, self.transcript]
            if mcfg.a2fc > 0:
                cost = cost - mcfg.a2fc * self.a2f_soft_iou(a2f_attn, self.onehot_seg_label)
            cost = cost.double().cpu().numpy()
        if mcfg.match == "o2o":
            ai, si = linear_sum_assignment(cost)
        elif mcfg.match == "o2m":
            ai, si = self._one_to_many_match(cost)
        else:
            raise ValueError(mcfg.match)
        ai = torch.as_tensor(np.asarray(ai), dtype=torch.int64)
        si = torch.as_tensor(np.asarray(si), dtype=torch.int64)
        self._match_cache = (ai, si, _to_dev(ai, clogit.device), _to_dev(si, clogit.device))
        return ai, si

    def _dev_match(self, match, dev):
        """Device copies of the match indices (made once per match, not once per loss term)."""
        aind, sind = match
        mc = getattr(self, "_match_cache", None)
        if mc is not None and aind is mc[0] and sind is mc[1] and mc[2].device == dev:
            return mc[2], mc[3]
        return _to_dev(aind, dev), _to_dev(sind, dev)

    def _one_to_many_match(self, cost):
        """loss.py:155-193."""
        tr = self._transcript_np if getattr(self, "_transcript_np", None) is not None else self.transcript.cpu().numpy()
        return one_to_many_match(cost, tr)

    def action_token_loss(self, match, action_clogit, is_logit=True):
        """loss.py:195-207."""
        A, C = action_clogit.shape[0], action_clogit.shape[-1]
        dev = action_clogit.device
        aind, sind = self._dev_match(match, dev)
        tgt = torch.full((A,), C - 1, dtype=torch.int64, device=dev)
        tgt[aind] = self.transcript[sind]
        x = action_clogit.squeeze(1)
        if is_logit:
            return _weighted_xent(x, tgt, self.cweight)
        return F.nll_loss(x, tgt, weight=self.cweight)

    def _attn_xent(self, attn, frame_tgt, dim, denom):
        lp = torch.log_softmax(attn, dim=dim - 1)
        term = -lp * frame_tgt
        if self.sweight is not None:
            term = term * self.sweight                      # column i scaled by sweight[i] (loss.py:218-219)
        return term.sum() / denom

    def cross_attn_loss(self, match, attn, dim=None):
        """loss.py:209-222."""
        assert dim >= 1
        aind, sind = self._dev_match(match, attn.device)
        tgt = self.onehot_seg_label[:, sind]
        return self._attn_xent(attn[0, :, aind], tgt, dim, self.onehot_seg_label.sum())

    def cross_attn_loss_tdu(self, match, attn, tdu, dim=None):
        """loss.py:224-244."""
        assert dim >= 1
        aind, sind = self._dev_match(match, attn.device)
        z = _zoom(tdu, self.onehot_seg_label)
        return self._attn_xent(attn[0, :, aind], z[:, sind], dim, z.sum())

    # ---------------- fused forms (one HIP launch pair per term group; same values) ----------------
    def frame_terms(self, frame_clogit, ce_coef=1.0, sm_coef=0.0):
        """ce_coef * frame_loss(frame_clogit) + sm_coef * smooth_loss(frame_clogit^T)
        (loss.py:246-258 and 8-18 on the same logits) as one fused term."""
        x = frame_clogit.squeeze(1) if frame_clogit.dim() == 3 else frame_clogit
        if not x.is_cuda:
            return ce_coef * self.frame_loss(x) + sm_coef * smooth_loss(x.unsqueeze(0))
        R, C = x.shape
        c_sm = (sm_coef / ((R - 1) * C) if R > 1 else float("inf")) if sm_coef else 0.0
        return fxf.ClassLossFn.apply(x, self.class_label.to(torch.int64).contiguous(), None, self.cweight[:C],
                                     ce_coef / float(R), c_sm)

    def seg_terms(self, seg_clogit, tdu, ce_coef=1.0):
        """ce_coef * frame_loss_tdu(seg_clogit, tdu) (loss.py:260-277) as one fused term."""
        x = seg_clogit.squeeze(1) if seg_clogit.dim() == 3 else seg_clogit
        if not x.is_cuda:
            return ce_coef * self.frame_loss_tdu(seg_clogit, tdu)
        z = _zoom(tdu, self.onehot_class_label).contiguous()
        return fxf.ClassLossFn.apply(x, None, z, self.cweight[:x.shape[1]], ce_coef / float(x.shape[0]), 0.0)

    def attn_terms(self, match, attn, axis, tdu=None, xe_coef=1.0, sm_coef=0.0):
        """xe_coef * cross_attn_loss(_tdu)(match, attn) + sm_coef * smooth_loss(attn) (loss.py:209-244,
        8-18) as one fused term.  ``attn`` is the (1, R, Q) logit view the reference passes;
        ``axis`` = dim - 1 of the reference call."""
        L = attn[0]
        aind, sind = match
        K = int(aind.numel())
        swn = getattr(self, "_sweight_np", None)
        if (not L.is_cuda) or swn is None or K > 64:
            z = None if tdu is None else _zoom(tdu, self.onehot_seg_label)
            xe = (self.cross_attn_loss(match, attn, dim=axis + 1) if tdu is None else
                  self.cross_attn_loss_tdu(match, attn, tdu, dim=axis + 1))
            return xe_coef * xe + (sm_coef * smooth_loss(attn) if sm_coef else 0.0)
        if len(swn) not in (K, 1):
            raise RuntimeError(f"cross_attn_loss: {K} matched columns vs {len(swn)} segment weights")
        sw = [float(swn[i if len(swn) == K else 0]) for i in range(K)]
        if tdu is None:
            z, denom = self.onehot_seg_label, float(L.shape[0])
        else:
            z, denom = _zoom(tdu, self.onehot_seg_label), float(tdu.num_seg)
        R, Q = L.shape
        c_sm = (sm_coef / ((R - 1) * Q) if R > 1 else float("inf")) if sm_coef else 0.0
        return fxf.AttnLossFn.apply(L, z.contiguous(), aind.tolist(), sind.tolist(), sw, axis, xe_coef / denom, c_sm)

    def frame_loss(self, frame_clogit, is_logit=True):
        """loss.py:246-258."""
        lp = torch.log_softmax(frame_clogit, dim=-1) if is_logit else frame_clogit
        w = self.cweight[:frame_clogit.shape[-1]]
        return (-lp * self.onehot_class_label * w).sum() / self.onehot_class_label.sum()

    def frame_loss_tdu(self, seg_clogit, tdu, is_logit=True):
        """loss.py:260-277."""
        x = seg_clogit.squeeze(1)
        lp = torch.log_softmax(x, dim=-1) if is_logit else x
        z = _zoom(tdu, self.onehot_class_label)
        w = self.cweight[:lp.shape[-1]]
        return (-lp * z * w).sum() / z.sum()


def infonce_contrastive_loss(projected_embeddings, text_embeddings, labels, temperature=0.07):
    """loss.py:280-341: (frame->text CE + per-class text->frame log-softmax) / 2."""
    T, B, D = projected_embeddings.shape
    emb = projected_embeddings.reshape(-1, D)
    lab = labels.reshape(-1)
    if lab.shape[0] != emb.shape[0]:
        lab = lab.repeat(B)
    n = text_embeddings.shape[0]
    if emb.is_cuda:
        sim = fxf.linear(emb, text_embeddings.detach(), None) * (1.0 / temperature)
    else:
        sim = emb @ text_embeddings.t() / temperature
    v2t = F.cross_entropy(sim, lab)
    tgt = F.one_hot(lab, num_classes=n).float()
    lp_t = F.log_softmax(sim.t(), dim=1)
    counts = torch.clamp(tgt.sum(0), min=1.0)
    t2v = (-(lp_t * tgt.t()).sum(1) / counts).mean()
    return (v2t + t2v) / 2.0


def one_to_many_match(cost, tr):
    """MatchCriterion._one_to_many_match (loss.py:155-193) on a host cost matrix (tokens x segments)
    and the segments' classes ``tr``."""
    actions = np.unique(tr)
    per_action = np.stack([cost[:, tr == a].sum(1) for a in actions], axis=1)
    aid, cid = linear_sum_assignment(per_action)
    rest = [a for a in range(cost.shape[0]) if a not in set(aid.tolist())]
    rest_c = per_action[rest].argmin(1) if rest else np.zeros(0, dtype=np.int64)
    token_cls = np.zeros(cost.shape[0])
    token_cls[np.array(aid.tolist() + rest, dtype=np.int64)] = np.array(
        [actions[i] for i in cid.tolist() + list(rest_c)])
    pairs = {}
    for a in actions:
        segs = np.where(tr == a)[0]
        toks = np.where(token_cls == a)[0]
        pick = cost[toks][:, segs].argmin(0)
        for s, k in zip(segs, pick):
            pairs[s] = toks[k]
    return list(pairs.values()), list(pairs.keys())
