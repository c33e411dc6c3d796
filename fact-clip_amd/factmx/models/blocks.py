"""FACT / FACT_CLIP with the reference's Python surface (fact_clip/models/blocks.py).

Same constructors, attribute names read by losses / eval / scripts
(``frame_clogit``, ``action_clogit``, ``a2f_attn``, ``f2a_attn``,
``*_attn_logit``, ``seg_clogit``, ``tdu``, ``action_feature``,
``projected_frame_embeddings``, ``fact_loss``, ``contrastive_loss``),
state_dict keys and ``forward(seq_list, label_list, compute_loss)``
contract.  Compute runs on the HIP kernels through factmx.functional.
"""
import torch
import torch.nn as nn

from .. import functional as fxf
from ..configs.utils import update_from
from ..dp import mark_block_input, mark_block_part
from ..utils import utils
from . import basic
from . import loss as loss_mod
from . import vloss
from .basic import time_mask, torch_class_label_to_segment_label
from .loss import MatchCriterion


def _frame_pos(pe_module, seq):
    """frame_pe(seq) (blocks.py:59/613); None when the table is empty (fpos=False), which is
    numerically identical to adding zeros and lets the kernels skip the add."""
    return None if pe_module.empty else pe_module(seq)


class FeatureProjection(nn.Module):
    """blocks.py:141-175: Linear -> LayerNorm -> ReLU -> Dropout -> Linear -> L2-normalise."""

    def __init__(self, feature_dim, clip_dim=512, hidden_dim=512, dropout=0.1):
        super().__init__()
        self.feature_dim = feature_dim
        self.clip_dim = clip_dim
        self.projection = nn.Sequential(nn.Linear(feature_dim, hidden_dim), nn.LayerNorm(hidden_dim), nn.ReLU(),
                                        nn.Dropout(dropout), nn.Linear(hidden_dim, clip_dim))

    def forward(self, feature):
        lin0, ln, _, drop, lin1 = self.projection
        shp = feature.shape
        h = fxf.linear_any_k(feature, lin0.weight, lin0.bias)
        h = fxf.layer_norm(h, ln.weight, ln.bias, ln.eps, relu=True)
        h = basic._dropout(h, drop.p, self.training)
        h = fxf.linear(h, lin1.weight, lin1.bias)
        y = fxf.l2_normalize(h)
        return y.reshape(*shp[:-1], self.clip_dim)


def _set_side(blk, rec):
    """setattr(blk, k, v) for the per-video side-channel values, straight into the instance dict (the
    lazily evaluated ones under their property's key): nn.Module.__setattr__ costs ~3 us a call and a
    step restores ~30 of them on the host's critical path."""
    d = blk.__dict__
    for k, val in rec.items():
        d[_LAZY_KEYS.get(k, k)] = val


class _Lazy:
    """A side-channel value computed on first read (frame-level gathers of segment attention that
    only evaluation code reads)."""
    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn


_LAZY_KEYS = {}


def _lazy_attr(name):
    key = "_lz_" + name
    _LAZY_KEYS[name] = key

    def get(self):
        d = self.__dict__
        if key not in d:
            raise AttributeError(name)
        v = d[key]
        if isinstance(v, _Lazy):
            v = d[key] = v.fn()
        return v

    def put(self, v):
        self.__dict__[key] = v
    return property(get, put)


class Block(nn.Module):
    """blocks.py:180-281."""

    f2a_attn = _lazy_attr("f2a_attn")
    a2f_attn = _lazy_attr("a2f_attn")

    def __repr__(self):
        return (f"{type(self).__name__}(\n  f:{self.frame_branch},\n  a:{self.action_branch},\n"
                f"  a2f:{getattr(self, 'a2f_layer', None)},\n  f2a:{getattr(self, 'f2a_layer', None)}\n)")

    def process_feature(self, feature, nclass):
        out, clogit = fxf.process_feature(feature, nclass)
        return out.unsqueeze(1), clogit.unsqueeze(1)

    def create_fbranch(self, cfg, in_dim=None, f_inmap=False):
        if in_dim is None:
            in_dim = cfg.f_dim
        if cfg.f == "m":
            return basic.MSTCN(in_dim, cfg.f_dim, cfg.hid_dim, cfg.f_layers, dropout=cfg.dropout, ln=cfg.f_ln,
                               ngroup=cfg.f_ngp, in_map=f_inmap)
        if cfg.f == "m2":
            return basic.MSTCN2(in_dim, cfg.f_dim, cfg.hid_dim, cfg.f_layers, dropout=cfg.dropout, ln=cfg.f_ln,
                                ngroup=cfg.f_ngp, in_map=f_inmap)
        raise ValueError(f"frame branch type {cfg.f!r} (the reference builds only 'm' / 'm2')")

    def create_abranch(self, cfg):
        if cfg.a == "sa":
            layer = basic.SALayer(cfg.a_dim, cfg.a_nhead, dim_feedforward=cfg.a_ffdim, dropout=cfg.dropout,
                                  attn_dropout=cfg.dropout)
            return basic.SADecoder(cfg.a_dim, cfg.a_dim, cfg.hid_dim, layer, cfg.a_layers, in_map=False)
        if cfg.a == "sca":
            layer = basic.SCALayer(cfg.a_dim, cfg.hid_dim, cfg.a_nhead, cfg.a_ffdim, dropout=cfg.dropout,
                                   attn_dropout=cfg.dropout)
            norm = torch.nn.LayerNorm(cfg.a_dim)
            return basic.SCADecoder(cfg.a_dim, cfg.a_dim, cfg.hid_dim, layer, cfg.a_layers, norm=norm, in_map=False)
        if cfg.a in ("gru", "gru_om"):
            assert self.cfg.FACT.trans
            return basic.ActionUpdate_GRU(cfg.a_dim, cfg.a_dim, cfg.hid_dim, cfg.a_layers, dropout=cfg.dropout,
                                          out_map=(cfg.a == "gru_om"))
        raise ValueError(cfg.a)

    def create_cross_attention(self, cfg, outdim, kq_pos=True):
        return basic.X2Y_map(cfg.hid_dim, cfg.hid_dim, outdim, head_dim=cfg.hid_dim, dropout=cfg.dropout,
                             kq_pos=kq_pos)

    @staticmethod
    def _abranch_prob(action_clogit, a2f_attn):
        """Per-frame class distribution of the most-attended non-null token (blocks.py:246-258),
        without a host sync: null tokens are masked to -inf before the argmax (first maximum, as
        the reference's argmax over the non-null subset).  Returns (prob (T, C), any_token)
        where ``any_token`` is a device bool: False is the reference's ``len(action_loc) == 0``."""
        acl = action_clogit.squeeze(1)
        a2f = a2f_attn.squeeze(0)
        null_cid = acl.shape[-1] - 1
        is_tok = acl.argmax(1) != null_cid
        masked = torch.where(is_tok[None, :], a2f, torch.full((), float("-inf"), device=a2f.device, dtype=a2f.dtype))
        qtk_prob = torch.softmax(acl[:, :-1], dim=1)
        return qtk_prob[masked.argmax(-1)], is_tok.any()

    @staticmethod
    def _eval(action_clogit, a2f_attn, frame_clogit, weight):
        fprob = torch.softmax(frame_clogit.squeeze(1), dim=-1)
        ab, any_tok = Block._abranch_prob(action_clogit, a2f_attn)
        mixed = ((1 - weight) * ab + weight * fprob).argmax(1)
        return torch.where(any_tok, mixed, fprob.argmax(1))

    @staticmethod
    def _eval_w_transcript(transcript, a2f_attn, frame_clogit, weight):
        fprob = torch.softmax(frame_clogit.squeeze(1), dim=-1)[:, transcript]
        n = len(transcript)
        aprob = torch.softmax(a2f_attn[0, :, :n], dim=-1)
        return transcript[((1 - weight) * aprob + weight * fprob).argmax(1)]

    def eval(self, transcript=None):
        if not self.cfg.FACT.trans:
            return self._eval(self.action_clogit, self.a2f_attn, self.frame_clogit, self.cfg.FACT.mwt)
        return self._eval_w_transcript(transcript, self.a2f_attn, self.frame_clogit, self.cfg.FACT.mwt)


def _frame_branch_batch(branch, f, vb):
    """The frame branch over vb.nvid stacked videos: MS-TCN and MS-TCN++ (MSTCN2) each as one fused
    stack call with per-video zero padding (ragged lengths through the row offsets)."""
    so = vb.f_off if vb.ragged else None
    if isinstance(branch, basic.MSTCN2):
        return fxf._2d(branch(f, T=vb.T, seq_off=so))
    return fxf.mstcn(branch, f, T=vb.T or 0, nvid=vb.nvid, seq_off=so)


class InputBlock(Block):
    """blocks.py:284-320."""

    # data parallelism: the action branch's gradient bucket launches from a hook on the frame-branch
    # output (the block's own input is the data: no gradient, no block hook), factmx.dp.mark_block_part
    dp_parts = ("action_branch",)

    def _dp_mark(self, f):
        ctx = self.__dict__.get("_dp_ctx")
        if ctx is not None:
            mark_block_part(ctx[0], ctx[1], "action_branch", f)

    def __init__(self, cfg, in_dim, nclass):
        super().__init__()
        self.cfg = cfg
        self.nclass = nclass
        bcfg = cfg.Bi
        self.frame_branch = self.create_fbranch(bcfg, in_dim, f_inmap=True)
        self.action_branch = self.create_abranch(bcfg)

    def forward(self, frame_feature, action_feature, frame_pos, action_pos, action_clogit=None):
        frame_feature = self.frame_branch(frame_feature)
        self._dp_mark(frame_feature)
        frame_feature, frame_clogit = self.process_feature(frame_feature, self.nclass)
        action_feature = self.action_branch(action_feature, frame_feature, pos=frame_pos, query_pos=action_pos)
        action_feature, action_clogit = self.process_feature(action_feature, self.nclass + 1)
        self.frame_clogit = frame_clogit
        self.action_clogit = action_clogit
        self.action_feature = action_feature[:, :, :-(self.nclass + 1)]
        return frame_feature, action_feature

    def forward_batch(self, f2, a2, fpos, apos, vb):
        """``forward`` over vb.nvid stacked videos (frames (nvid*T, C), tokens (nvid*Q, A));
        per-video side-channel attributes go to ``self._vrec``."""
        f = _frame_branch_batch(self.frame_branch, f2, vb)
        self._dp_mark(f)
        f_out, f_cl = fxf.process_feature(f, self.nclass)
        a = fxf.decoder(self.action_branch, a2, f_out, pos=fpos, query_pos=apos, nvid=vb.nvid,
                        mem_off=vb.f_off if vb.ragged else None)
        a_out, a_cl = fxf.process_feature(a, self.nclass + 1)
        n = self.nclass + 1
        fc, ac, ao = vb.frames(f_cl), vb.tokens(a_cl), vb.tokens(a_out)
        self._vrec = [dict(frame_clogit=fc[v].unsqueeze(1), action_clogit=ac[v].unsqueeze(1),
                           action_feature=ao[v][:, :-n].unsqueeze(1)) for v in range(vb.nvid)]
        self.__dict__["_bt"] = dict(f_cl=f_cl, a_cl=a_cl)
        return f_out, a_out

    def compute_loss(self, criterion, match=None):
        """blocks.py:313-320: frame CE + token CE + sw * smooth(frame logits); the frame CE and its
        smooth term are one fused kernel pair."""
        atk = criterion.action_token_loss(match, self.action_clogit)
        return criterion.frame_terms(self.frame_clogit, 1.0, self.cfg.Loss.sw) + atk


class UpdateBlock(Block):
    """blocks.py:322-382."""

    def __init__(self, cfg, nclass):
        super().__init__()
        self.cfg = cfg
        self.nclass = nclass
        bcfg = cfg.Bu
        self.frame_branch = self.create_fbranch(bcfg)
        self.f2a_layer = self.create_cross_attention(bcfg, bcfg.a_dim)
        self.action_branch = self.create_abranch(bcfg)
        self.a2f_layer = self.create_cross_attention(bcfg, bcfg.f_dim)

    def forward(self, frame_feature, action_feature, frame_pos, action_pos):
        action_feature = self.f2a_layer(frame_feature, action_feature, X_pos=frame_pos, Y_pos=action_pos)
        action_feature = self.action_branch(action_feature, action_pos)
        action_feature, action_clogit = self.process_feature(action_feature, self.nclass + 1)
        frame_feature = self.a2f_layer(action_feature, frame_feature, X_pos=action_pos, Y_pos=frame_pos)
        frame_feature = self.frame_branch(frame_feature)
        frame_feature, frame_clogit = self.process_feature(frame_feature, self.nclass)
        self.frame_clogit = frame_clogit
        self.action_clogit = action_clogit
        self.action_feature = action_feature[:, :, :-(self.nclass + 1)]
        self.f2a_attn = self.f2a_layer.attn[0]
        self.a2f_attn = self.a2f_layer.attn[0]
        self.f2a_attn_logit = self.f2a_layer.attn_logit.squeeze(0).unsqueeze(0)
        self.a2f_attn_logit = self.a2f_layer.attn_logit.squeeze(0).unsqueeze(0)
        return frame_feature, action_feature

    def forward_batch(self, f2, a2, fpos, apos, vb):
        f2a, a2f = self.f2a_layer, self.a2f_layer
        a, f2a_lg, f2a_at = fxf.x2y(f2a, f2, a2, fpos if f2a.kq_pos else None, apos if f2a.kq_pos else None,
                                    rows=(vb.f_off, vb.a_off))
        a = fxf.decoder(self.action_branch, a, None, query_pos=apos, nvid=vb.nvid)
        a_out, a_cl = fxf.process_feature(a, self.nclass + 1)
        f, a2f_lg, a2f_at = fxf.x2y(a2f, a_out, f2, apos if a2f.kq_pos else None, fpos if a2f.kq_pos else None,
                                    rows=(vb.a_off, vb.f_off))
        f = _frame_branch_batch(self.frame_branch, f, vb)
        if vb.on_a2f is not None and vb.last is self:
            # the loss phase's matching starts here (vloss.EarlyMatch): its host work runs while the
            # device works through the frame branch just issued, its cost launch queues behind it
            vb.on_a2f(vb, a_cl, a2f_at)
        f_out, f_cl = fxf.process_feature(f, self.nclass)
        n, Q = self.nclass + 1, vb.Q
        recs = []
        fc, ac, ao = vb.frames(f_cl), vb.tokens(a_cl), vb.tokens(a_out)
        qt = [Q * T for T in vb.Ts]
        fat, aat, flg, alg = (torch.split(t, qt) for t in (f2a_at, a2f_at, f2a_lg, a2f_lg))
        for v in range(vb.nvid):
            T = vb.Ts[v]
            recs.append(dict(frame_clogit=fc[v].unsqueeze(1), action_clogit=ac[v].unsqueeze(1),
                             action_feature=ao[v][:, :-n].unsqueeze(1),
                             f2a_attn=fat[v].view(1, Q, T), a2f_attn=aat[v].view(1, T, Q),
                             f2a_attn_logit=flg[v].view(1, Q, T), a2f_attn_logit=alg[v].view(1, T, Q)))
        self.__dict__["_vrec"] = recs     # (plain attributes: no nn.Module.__setattr__ walk)
        self.__dict__["_bt"] = dict(f_cl=f_cl, a_cl=a_cl, f2a_lg=f2a_lg, a2f_lg=a2f_lg, a2f_at=a2f_at)
        return f_out, a_out

    def compute_loss(self, criterion, match=None):
        """blocks.py:369-382: token CE + f2a / a2f cross-attention CE + frame CE + sw * (smooth of both
        attention logits and the frame logits), as three fused terms + the token CE."""
        sw = self.cfg.Loss.sw
        atk = criterion.action_token_loss(match, self.action_clogit)
        f2a_t = self.f2a_attn_logit.transpose(1, 2)
        f2a = criterion.attn_terms(match, f2a_t, axis=0, xe_coef=1.0, sm_coef=sw)
        a2f = criterion.attn_terms(match, self.a2f_attn_logit, axis=1, xe_coef=1.0, sm_coef=sw)
        return _sum_terms([atk, f2a, a2f, criterion.frame_terms(self.frame_clogit, 1.0, sw)])


class UpdateBlockTDU(Block):
    """blocks.py:385-497: segment-level update with device-side temporal down/up-sampling."""

    def __init__(self, cfg, nclass):
        super().__init__()
        self.cfg = cfg
        self.nclass = nclass
        bcfg = cfg.BU
        self.frame_branch = self.create_fbranch(bcfg)
        self.seg_update = nn.GRU(bcfg.hid_dim, bcfg.hid_dim // 2, bcfg.s_layers, bidirectional=True)
        self.seg_combine = nn.Linear(bcfg.hid_dim, bcfg.hid_dim)
        self.f2a_layer = self.create_cross_attention(bcfg, bcfg.a_dim)
        self.action_branch = self.create_abranch(bcfg)
        self.a2f_layer = self.create_cross_attention(bcfg, bcfg.f_dim)
        self.sf_merge = nn.Sequential(nn.Linear(bcfg.hid_dim + bcfg.f_dim, bcfg.f_dim), nn.ReLU())

    def temporal_downsample(self, frame_feature):
        f2 = fxf._2d(frame_feature)
        tdu = basic.TemporalDownsampleUpsample.from_probs(f2, f2.shape[1] - self.nclass, self.nclass)
        seg = tdu.feature_frame2seg(frame_feature)
        seg = fxf.gru(self.seg_update, seg, relu=True)      # relu(seg_update(seg)) (blocks.py:432)
        seg = fxf.linear(seg, self.seg_combine.weight, self.seg_combine.bias).unsqueeze(1)
        seg, seg_clogit = self.process_feature(seg, self.nclass)
        return tdu, seg, seg_clogit

    def temporal_upsample(self, tdu, seg_feature, frame_feature):
        lin = self.sf_merge[0]
        y = fxf.SegMergeFn.apply(fxf._2d(seg_feature), fxf._2d(frame_feature), tdu.seg_id32, tdu.start32, tdu.end32,
                                 lin.weight, lin.bias)
        return y.unsqueeze(1)

    def forward(self, frame_feature, action_feature, frame_pos, action_pos):
        tdu, seg_feature, seg_clogit = self.temporal_downsample(frame_feature)
        seg_pos = None if frame_pos is None else frame_pos[tdu.centers()]
        action_feature = self.f2a_layer(seg_feature, action_feature, X_pos=seg_pos, Y_pos=action_pos)
        action_feature = self.action_branch(action_feature, action_pos)
        action_feature, action_clogit = self.process_feature(action_feature, self.nclass + 1)
        seg_feature = self.a2f_layer(action_feature, seg_feature, X_pos=action_pos, Y_pos=seg_pos)
        frame_feature = self.temporal_upsample(tdu, seg_feature, frame_feature)
        frame_feature = self.frame_branch(frame_feature)
        frame_feature, frame_clogit = self.process_feature(frame_feature, self.nclass)
        self.frame_clogit = frame_clogit
        self.seg_clogit = seg_clogit
        self.tdu = tdu
        self.action_clogit = action_clogit
        self.action_feature = action_feature[:, :, :-(self.nclass + 1)]
        self.f2a_attn_logit = self.f2a_layer.attn_logit.squeeze(0).unsqueeze(0)
        self.f2a_attn = tdu.attn_seg2frame(self.f2a_layer.attn[0].transpose(2, 1)).transpose(2, 1)
        self.a2f_attn_logit = self.a2f_layer.attn_logit.squeeze(0).unsqueeze(0)
        self.a2f_attn = tdu.attn_seg2frame(self.a2f_layer.attn[0])
        return frame_feature, action_feature

    def forward_batch(self, f2, a2, fpos, apos, vb):
        # temporal downsample: one segmentation launch + ONE host read of every video's S
        # (the first TDU block: the loss phase's label-only host work runs while the host waits for S)
        hook, vb.while_waiting = vb.while_waiting, None
        S, local, (gid, gst, gen) = fxf.segments_from_probs_batched(f2, f2.shape[1] - self.nclass, self.nclass,
                                                                     vb.f_off, hook)
        s_off = [0]
        for n_ in S:
            s_off.append(s_off[-1] + n_)
        tdus = [basic.TemporalDownsampleUpsample(*local[v]) for v in range(vb.nvid)]
        seg = fxf.SegMeanFn.apply(f2, gid, gst, gen)
        seg = fxf.gru(self.seg_update, seg, seq_off=s_off, relu=True)     # relu folded into the kernel
        seg = fxf.linear(seg, self.seg_combine.weight, self.seg_combine.bias)
        seg_out, seg_cl = fxf.process_feature(seg, self.nclass)
        seg_pos = None
        if fpos is not None:
            seg_pos = fpos[torch.div(gst + gen, 2, rounding_mode="floor").to(torch.int64)]
        f2a, a2f = self.f2a_layer, self.a2f_layer
        a, f2a_lg, f2a_at = fxf.x2y(f2a, seg_out, a2, seg_pos if f2a.kq_pos else None, apos if f2a.kq_pos else None,
                                    rows=(s_off, vb.a_off))
        a = fxf.decoder(self.action_branch, a, None, query_pos=apos, nvid=vb.nvid)
        a_out, a_cl = fxf.process_feature(a, self.nclass + 1)
        sg, a2f_lg, a2f_at = fxf.x2y(a2f, a_out, seg_out, apos if a2f.kq_pos else None,
                                     seg_pos if a2f.kq_pos else None, rows=(vb.a_off, s_off))
        lin = self.sf_merge[0]
        f = fxf.SegMergeFn.apply(sg, f2, gid, gst, gen, lin.weight, lin.bias)
        f = _frame_branch_batch(self.frame_branch, f, vb)
        if vb.on_a2f is not None and vb.last is self:
            vb.on_a2f(vb, a_cl, a2f_at, (s_off, local))     # (see UpdateBlock.forward_batch)
        f_out, f_cl = fxf.process_feature(f, self.nclass)
        n, Q = self.nclass + 1, vb.Q
        recs = []
        fc, ac, ao = vb.frames(f_cl), vb.tokens(a_cl), vb.tokens(a_out)
        sc = torch.split(seg_cl, [s_off[v + 1] - s_off[v] for v in range(vb.nvid)])
        qs = [Q * S[v] for v in range(vb.nvid)]
        fat, aat, flg, alg = (torch.split(t, qs) for t in (f2a_at, a2f_at, f2a_lg, a2f_lg))
        for v in range(vb.nvid):
            Sv, tdu = S[v], tdus[v]
            f2a_at_v = fat[v].view(1, 1, Q, Sv)
            a2f_at_v = aat[v].view(1, 1, Sv, Q)
            recs.append(dict(frame_clogit=fc[v].unsqueeze(1),
                             seg_clogit=sc[v].unsqueeze(1), tdu=tdu,
                             action_clogit=ac[v].unsqueeze(1),
                             action_feature=ao[v][:, :-n].unsqueeze(1),
                             f2a_attn_logit=flg[v].view(1, Q, Sv),
                             f2a_attn=_Lazy(lambda t=tdu, a=f2a_at_v: t.attn_seg2frame(a[0].transpose(2, 1))
                                            .transpose(2, 1)),
                             a2f_attn_logit=alg[v].view(1, Sv, Q),
                             a2f_attn=_Lazy(lambda t=tdu, a=a2f_at_v: t.attn_seg2frame(a[0]))))
        self.__dict__["_vrec"] = recs     # (plain attributes: no nn.Module.__setattr__ walk)
        self.__dict__["_bt"] = dict(f_cl=f_cl, a_cl=a_cl, f2a_lg=f2a_lg, a2f_lg=a2f_lg, a2f_at=a2f_at, seg_cl=seg_cl, S=S,
                        s_off=s_off, local=local)
        return f_out, a_out

    def compute_loss(self, criterion, match=None):
        """blocks.py:487-497: (frame CE + segment CE) / 2 + token CE + segment-level f2a / a2f
        cross-attention CE + sw * smooth(frame logits), as four fused terms + the token CE."""
        atk = criterion.action_token_loss(match, self.action_clogit)
        f2a = criterion.attn_terms(match, self.f2a_attn_logit.transpose(1, 2), axis=0, tdu=self.tdu)
        a2f = criterion.attn_terms(match, self.a2f_attn_logit, axis=1, tdu=self.tdu)
        return _sum_terms([criterion.frame_terms(self.frame_clogit, 0.5, self.cfg.Loss.sw),
                           criterion.seg_terms(self.seg_clogit, self.tdu, 0.5), atk, f2a, a2f])


def _build_blocks(cfg, in_dim, n_classes):
    base = cfg.Bi
    blocks = []
    for t in cfg.FACT.block:
        if t == "i":
            blocks.append(InputBlock(cfg, in_dim, n_classes))
        elif t == "u":
            update_from(cfg.Bu, base, inplace=True)
            base = cfg.Bu
            blocks.append(UpdateBlock(cfg, n_classes))
        elif t == "U":
            update_from(cfg.BU, base, inplace=True)
            base = cfg.BU
            blocks.append(UpdateBlockTDU(cfg, n_classes))
        else:
            raise ValueError(t)
    return nn.ModuleList(blocks)


class _OutRef:
    """Element(s) of the fused loss output vector, indexed on first read (vloss.run: selecting every
    side-channel value at the end of the forward costs ~0.1 ms of host time on the critical path)."""
    __slots__ = ("out", "idx")

    def __init__(self, out, idx):
        self.out, self.idx = out, idx

    def get(self):
        return [self.out[i] for i in self.idx] if isinstance(self.idx, list) else self.out[self.idx]


def _lazy_out_attr(name):
    key = "_lo_" + name

    def get(self):
        d = self.__dict__
        if key not in d:
            raise AttributeError(name)
        v = d[key]
        if isinstance(v, _OutRef):
            v = d[key] = v.get()
        return v

    def put(self, v):
        self.__dict__[key] = v
    return property(get, put)


class _FACTBase(nn.Module):
    # side-channel loss values of the last forward (blocks.py:905-910); the fused loss phase stores
    # _OutRef placeholders that resolve on first read
    loss_list = _lazy_out_attr("loss_list")
    fact_loss = _lazy_out_attr("fact_loss")
    contrastive_loss = _lazy_out_attr("contrastive_loss")

    def _init_common(self, cfg, n_classes):
        self.cfg = cfg
        self.num_classes = n_classes
        bcfg = cfg.Bi
        self.frame_pe = basic.PositionalEncoding(bcfg.hid_dim, max_len=10000, empty=(not cfg.FACT.fpos))
        self.channel_masking_dropout = nn.Dropout2d(p=cfg.FACT.cmr)
        if not cfg.FACT.trans:
            self.action_query = nn.Parameter(torch.randn([cfg.FACT.ntoken, 1, bcfg.a_dim]))
        else:
            self.action_pe = basic.PositionalEncoding(bcfg.a_dim, max_len=1000)
            self.action_embed = nn.Embedding(n_classes, bcfg.a_dim)

    def _run_blocks(self, seq, transcript):
        frame_feature = seq
        frame_pe = _frame_pos(self.frame_pe, seq)
        if self.cfg.FACT.cmr and self.training:
            frame_feature = self.channel_masking_dropout(frame_feature.permute([1, 2, 0])).permute([2, 0, 1])
        if self.cfg.TM.use and self.training:
            frame_feature = time_mask(frame_feature, self.cfg.TM.t, self.cfg.TM.m, self.cfg.TM.p,
                                      replace_with_zero=True)
        if not self.cfg.FACT.trans:
            action_pe = self.action_query
            action_feature = torch.zeros_like(action_pe)
        else:
            action_pe = self.action_pe(transcript)
            action_feature = self.action_embed(transcript).unsqueeze(1) + action_pe
            action_pe = torch.zeros_like(action_pe)
        block_output = []
        for k, block in enumerate(self.block_list):
            mark_block_input(self, k, frame_feature)
            block.__dict__["_dp_ctx"] = (self, k)      # (not a submodule registration)
            frame_feature, action_feature = block(frame_feature, action_feature, frame_pe, action_pe)
            block_output.append([frame_feature, action_feature])
        return block_output

    def _forward_batch(self, seq_list, on_a2f=None):
        """All videos through the blocks in lockstep (see _forward_videos); returns restore(v), which
        points every side-channel attribute at video v's views.  ``on_a2f`` (vloss.EarlyMatch) runs
        when the last block's token logits and token->frame attention exist."""
        nvid = len(seq_list)
        Q = self.cfg.FACT.ntoken
        vb = _VideoBatch(nvid, [int(s.shape[0]) for s in seq_list], Q)
        vb.on_a2f, vb.last = on_a2f, self.block_list[-1]
        if on_a2f is not None:
            dev = seq_list[0].device
            vb.while_waiting = lambda: on_a2f.prepare(dev)
        frames = []
        for seq in seq_list:
            x = seq.unsqueeze(1)
            if self.cfg.FACT.cmr and self.training:
                x = self.channel_masking_dropout(x.permute([1, 2, 0])).permute([2, 0, 1])
            if self.cfg.TM.use and self.training:
                x = time_mask(x, self.cfg.TM.t, self.cfg.TM.m, self.cfg.TM.p, replace_with_zero=True)
            frames.append(x.squeeze(1))
        f2 = torch.cat(frames, 0)
        fpe = [_frame_pos(self.frame_pe, s.unsqueeze(1)) for s in seq_list]
        fpos = None if fpe[0] is None else torch.cat([p.squeeze(1) for p in fpe], 0)
        # one shared gradient buffer for the query table's readers (fxf.PosGradSink: no pairwise adds)
        apos = fxf.pos_sink(self.action_query.squeeze(1).repeat(nvid, 1))
        a2 = torch.zeros_like(apos)
        for k, blk in enumerate(self.block_list):
            mark_block_input(self, k, f2)       # DP: block k's gradient bucket launches once f2 has its grad
            blk.__dict__["_dp_ctx"] = (self, k)
            f2, a2 = blk.forward_batch(f2, a2, fpos, apos, vb)
        proj = None
        if isinstance(self, FACT_CLIP):
            feat_dim = f2.shape[-1] - self.num_classes
            proj = self.frame_projection(f2[:, :feat_dim])

        self._proj = proj
        self._vb = vb
        proj_v = None if proj is None else vb.frames(proj)

        def restore(v):
            for blk in self.block_list:
                _set_side(blk, blk._vrec[v])
            if proj_v is not None:
                self.projected_frame_embeddings = proj_v[v].unsqueeze(1)
        return restore

    def _fact_loss(self, label, label_host=None):
        mc: MatchCriterion = self.mcriterion
        mc.set_label(label, label_host=label_host)
        last = self.block_list[-1]
        match = mc.match(basic.logit2prob(last.action_clogit, dim=-1), last.a2f_attn)
        self.loss_list = [blk.compute_loss(mc, match) for blk in self.block_list]
        return _sum_terms(self.loss_list) / len(self.loss_list)

    def save_model(self, fname):
        torch.save(self.state_dict(), fname)


class FACT(_FACTBase):
    """blocks.py:19-135 (vanilla FACT)."""

    def __init__(self, cfg, in_dim, n_classes):
        super().__init__()
        self._init_common(cfg, n_classes)
        self.block_list = _build_blocks(cfg, in_dim, n_classes)
        self.mcriterion = None

    def _forward_one_video(self, seq, transcript=None):
        return self._run_blocks(seq, transcript)

    def _loss_one_video(self, label, label_host=None):
        return self._fact_loss(label, label_host)

    def forward(self, seq_list, label_list, compute_loss=False):
        return _forward_videos(self, seq_list, label_list, compute_loss)


class FACT_CLIP(_FACTBase):
    """blocks.py:504-920: FACT + CLIP projection head + InfoNCE; zero-shot eval via text similarity."""

    # data parallelism: the projection head reads only the last block's output, so its gradients are
    # final once the backward is under way -- reduced with the first block bucket (factmx.dp)
    dp_head_modules = ("frame_projection",)

    def __init__(self, cfg, in_dim, n_classes, text_embeddings=None):
        super().__init__()
        self._init_common(cfg, n_classes)
        # feature width from Bi.hid_dim, evaluated before the block loop (blocks.py:568)
        frame_feature_dim = cfg.Bi.hid_dim - n_classes
        self.frame_projection = FeatureProjection(feature_dim=frame_feature_dim, clip_dim=512,
                                                  hidden_dim=cfg.CLIP.projection_hidden_dim,
                                                  dropout=cfg.CLIP.projection_dropout)
        if text_embeddings is not None:
            self.register_buffer("text_embeddings", text_embeddings)
        else:
            self.text_embeddings = None
        self.block_list = _build_blocks(cfg, in_dim, n_classes)
        self.mcriterion = None

    def _forward_one_video(self, seq, transcript=None):
        out = self._run_blocks(seq, transcript)
        frame_feature = out[-1][0]
        feat_dim = frame_feature.shape[-1] - self.num_classes
        self.projected_frame_embeddings = self.frame_projection(frame_feature[:, :, :feat_dim])
        return out

    def _loss_one_video(self, label, label_host=None):
        fact_loss = self._fact_loss(label, label_host)
        if self.text_embeddings is None or not hasattr(self, "projected_frame_embeddings"):
            return fact_loss
        mc = self.mcriterion
        text = self.text_embeddings
        labels = mc.class_label
        emb = self.projected_frame_embeddings
        hold = list(getattr(self.cfg, "holdout_classes", []) or [])
        if hold:
            n = text.shape[0]
            key = (n, tuple(hold), str(text.device))
            if getattr(self, "_holdout_key", None) != key:
                seen_h = [i for i in range(n) if i not in set(hold)]
                remap_h = torch.full((n,), -1, dtype=torch.long)
                remap_h[seen_h] = torch.arange(len(seen_h))
                self._holdout_key = key
                self._holdout_tabs = (torch.tensor(seen_h, device=text.device), remap_h.to(text.device),
                                      remap_h.numpy())
            seen, remap, remap_np = self._holdout_tabs
            text = text[seen]
            labels = remap[labels]
            lab_np = getattr(mc, "_label_np", None)
            if lab_np is not None:
                valid_np = remap_np[lab_np] != -1
                n_valid, all_valid = int(valid_np.sum()), bool(valid_np.all())
            else:                                     # no host copy: decide on the device (a sync)
                valid_d = labels != -1
                n_valid, all_valid = int(valid_d.sum()), bool(valid_d.all())
            if not all_valid:
                if n_valid == 0:
                    return fact_loss
                valid = labels != -1
                labels = labels[valid]
                emb = emb.reshape(-1, emb.shape[-1])[valid].unsqueeze(1)
        con = loss_mod.infonce_contrastive_loss(emb, text, labels, temperature=self.cfg.CLIP.temp)
        total = self.cfg.CLIP.fact_loss_weight * fact_loss + self.cfg.CLIP.contrastive_weight * con
        self.fact_loss = fact_loss
        self.contrastive_loss = con
        return total

    def eval_with_clip(self, transcript=None):
        """blocks.py:788-887."""
        if self.text_embeddings is None or not hasattr(self, "projected_frame_embeddings"):
            return self.block_list[-1].eval(transcript)
        emb = self.projected_frame_embeddings.squeeze(1)
        if emb.is_cuda:
            with torch.no_grad():
                logits = fxf.matmul_nt(emb.detach(), self.text_embeddings, alpha=1.0 / self.cfg.CLIP.temp)
        else:
            logits = emb @ self.text_embeddings.t() / self.cfg.CLIP.temp
        clip_prob = torch.softmax(logits, dim=-1)
        last = self.block_list[-1]
        ab, any_tok = Block._abranch_prob(last.action_clogit, last.a2f_attn)
        w = self.cfg.FACT.mwt
        return torch.where(any_tok, ((1 - w) * ab + w * clip_prob).argmax(1), clip_prob.argmax(1))

    def forward(self, seq_list, label_list, compute_loss=False):
        return _forward_videos(self, seq_list, label_list, compute_loss)


def _sum_terms(terms):
    """Sum of scalar loss terms in one reduction launch (a chain of `+` costs one 1-element kernel
    per term); Python floats (terms a config switched off) are added on the host side."""
    ts = [t for t in terms if torch.is_tensor(t)]
    const = sum(float(t) for t in terms if not torch.is_tensor(t))
    if not ts:
        return const
    total = ts[0] if len(ts) == 1 else torch.stack([t.reshape(()) for t in ts]).sum()
    return total + const if const else total


class _VideoBatch:
    """Row layout of nvid videos stacked for one batched pass: frames of video v are rows
    [f_off[v], f_off[v+1]) (lengths Ts, ragged allowed), its action tokens rows [v*Q, (v+1)*Q).
    T is the common length of an equal-length batch (None when ragged)."""

    def __init__(self, nvid, Ts, Q):
        self.nvid, self.Ts, self.Q = nvid, list(Ts), Q
        self.ragged = len(set(self.Ts)) > 1
        self.T = None if self.ragged else self.Ts[0]
        self.f_off = [0]
        for T in self.Ts:
            self.f_off.append(self.f_off[-1] + T)
        self.a_off = [v * Q for v in range(nvid + 1)]
        self.on_a2f = self.last = self.while_waiting = None

    def fr(self, v):
        return slice(self.f_off[v], self.f_off[v + 1])

    def tk(self, v):
        return slice(v * self.Q, (v + 1) * self.Q)

    # Per-video chunks through ONE split node per tensor: its backward concatenates the chunks'
    # gradients once, where per-video slicing costs a zero-filled full-size tensor, a copy and an
    # accumulating add per video (for every side-channel tensor a loss reads).
    def frames(self, t):
        return torch.split(t, self.Ts, dim=0)

    def tokens(self, t):
        return torch.split(t, self.Q, dim=0)


# lockstep batches take the loss phase through models/vloss.py (False: per-video MatchCriterion ops)
FUSED_LOSS = True


MAX_LOCKSTEP_VIDEOS = 16   # ragged frame-branch convs carry at most 16 video offsets per launch


def _batchable(net, seq_list):
    """The lockstep path (any video lengths, one video included) needs the fused decoders, GPU inputs
    and no transcript input."""
    if not seq_list or len(seq_list) > MAX_LOCKSTEP_VIDEOS or net.cfg.FACT.trans:
        return False
    if any(not s.is_cuda or s.shape[0] < 1 for s in seq_list):
        return False
    for blk in net.block_list:
        if not basic._fused_decoder_ok(blk.action_branch) or not hasattr(blk, "forward_batch"):
            return False
    return True


def _label_to_host(label):
    if label.is_cuda:
        label_host = label.to("cpu", non_blocking=True)
        ready = torch.cuda.Event()
        ready.record()
        return label_host, ready
    return label, None


def _forward_videos(net, seq_list, label_list, compute_loss):
    """FACT.forward / FACT_CLIP.forward (blocks.py:118-135, 889-917): per-video predictions and the
    mean of the per-video losses, with the reference's side-channel attributes holding the last
    video's values afterwards.

    Equal-length videos run in LOCKSTEP (``forward_batch``): every block processes all videos in one
    pass (frame GEMMs over nvid*T rows, token GEMMs over nvid*Q rows, attention kept within each
    video, one segmentation read-back per TDU block for all videos); the losses then run per video
    on that video's views.  Otherwise videos run one by one as in the reference.  Either way: the
    transcript is only built where it is used (FACT.trans), labels reach the host by an async copy
    started before the forward, predictions and loss floats come back in one read-back."""
    clip = isinstance(net, FACT_CLIP)
    vloss.resolve_pending()     # the previous step's read-back (raises a kernel failure it carried)
    hosts = [_label_to_host(l_) for l_ in label_list]
    save_list, losses, pending, preds = [], [], [], []

    def finish_video(v, trans):
        preds.append(net.eval_with_clip(trans) if clip else net.block_list[-1].eval(trans))
        save = {}
        save_list.append(save)
        if compute_loss:
            lo = net._loss_one_video(label_list[v], label_host=hosts[v])
            losses.append(lo)
            keys, vals = ["loss"], [lo.detach()]
            if clip and hasattr(net, "fact_loss"):
                keys.append("fact_loss")
                vals.append(net.fact_loss.detach().reshape(()))
            if clip and hasattr(net, "contrastive_loss"):
                keys.append("contrastive_loss")
                vals.append(net.contrastive_loss.detach().reshape(()))
            pending.append((save, keys, vals))

    net.video_segments = []     # per video: the TDU segment count of every U block (host ints, no sync)
    if _batchable(net, seq_list):
        fused = FUSED_LOSS and vloss.supported(net)
        early = vloss.EarlyMatch(net, hosts) if (fused and compute_loss) else None
        restore = net._forward_batch(seq_list, early)
        if fused:
            nvid = len(seq_list)
            restore(nvid - 1)       # side-channel attributes: the last video's views, as in the reference
            net.video_segments = [[blk._bt["S"][v] for blk in net.block_list if "S" in blk._bt]
                                  for v in range(nvid)]
            try:
                return vloss.run(net, net._vb, compute_loss, early)
            except vloss.TableTooLarge:
                # more matched columns than the fused term table holds (o2m past FX_LOSS_MAXK segments):
                # this batch's losses and predictions run per video on the lockstep outputs
                net.video_segments = []
        for v in range(len(seq_list)):
            restore(v)
            net.video_segments.append([blk.tdu.num_seg for blk in net.block_list if hasattr(blk, "tdu")])
            finish_video(v, None)
    else:
        for v, (seq, label) in enumerate(zip(seq_list, label_list)):
            trans = torch_class_label_to_segment_label(label)[0] if net.cfg.FACT.trans else None
            net._forward_one_video(seq.unsqueeze(1), trans)
            net.video_segments.append([blk.tdu.num_seg for blk in net.block_list if hasattr(blk, "tdu")])
            finish_video(v, trans)
    # one read-back for every video's predictions (+ loss floats)
    st = fxf._status.get(preds[0].device) if preds[0].is_cuda else None    # kernel-side failures (GRU timeout)
    host = torch.cat([p.reshape(-1).to(torch.int64) for p in preds] +
                     ([st[:1].to(torch.int64)] if st is not None else [])).cpu().numpy()
    if st is not None:
        fxf.status_raise(int(host[-1]), preds[0].device)
    off = 0
    for save, p in zip(save_list, preds):
        save["pred"] = host[off:off + p.numel()].copy()
        off += p.numel()
    if compute_loss:
        vals = torch.cat([v.float().reshape(1) for _, _, vs in pending for v in vs]).tolist()
        i = 0
        for save, keys, _ in pending:
            save["loss"] = dict(zip(keys, vals[i:i + len(keys)]))
            i += len(keys)
        return sum(losses) / len(losses), save_list
    return save_list
