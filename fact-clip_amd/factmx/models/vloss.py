"""The loss phase of a lockstep batch of videos in a handful of launches (blocks._forward_videos).

The reference computes, per video and one after another (blocks.py:118-135 / 889-917):
predictions (Block._eval / eval_with_clip, blocks.py:243-261, 788-887), the Hungarian matching
(MatchCriterion.match, loss.py:108-153, soft IoU 91-106), every block's loss terms (compute_loss,
blocks.py:313-320, 369-382, 487-497 over loss.py:195-277) and the CLIP InfoNCE term
(loss.py:280-341, blocks.py:677-786).  Here, for all videos at once:

  1. one upload of the host-side tables (ground-truth segments from the labels, class weights,
     the per-video pointer table), then ONE launch of per-frame predictions (fx_eval_pred, after
     the CLIP similarity GEMM) and ONE launch of every video's matching cost (fx_match_cost);
  2. one read-back (predictions + costs), the Hungarian assignment per video on the host (scipy,
     as the reference);
  3. one upload of the term table (every CE / smooth / cross-attention / InfoNCE term of every
     block of every video, soft targets described by frame intervals instead of one-hot / "zoom"
     matrices), and fx_loss_terms_fwd: class terms, attention terms, InfoNCE, fixed-order finish
     and one combine into [batch loss, per video (loss, fact, contrastive, per-block values)].
     The backward (fx_loss_terms_bwd) writes the gradient of every logit tensor in four launches.
"""
import ctypes
import os

import numpy as np
import torch
from scipy.optimize import linear_sum_assignment

from .. import functional as fxf
from .. import native as nx
from .loss import one_to_many_match


class _Pack:
    """Host tables and ABI structs laid out in one buffer: allocated on the device first (so the
    structs can hold device addresses), then filled on the host and sent by ONE non-blocking copy
    from pinned memory."""

    def __init__(self):
        self.items = []
        self.size = 0

    def _reserve(self, nbytes):
        off = (self.size + 15) & ~15
        self.size = off + max(int(nbytes), 4)
        return off

    def array(self, a, dtype):
        a = np.ascontiguousarray(a, dtype=dtype).reshape(-1)
        off = self._reserve(a.nbytes)
        self.items.append((off, a))
        return off

    def structs(self, ctype, n):
        arr = (ctype * n)()
        off = self._reserve(ctypes.sizeof(arr))
        self.items.append((off, arr))
        return off, arr

    def alloc(self, dev):
        self.dev = torch.empty(self.size, dtype=torch.uint8, device=dev)
        self.base = self.dev.data_ptr()
        return self.base

    def send(self):
        host = torch.empty(self.size, dtype=torch.uint8, pin_memory=True)
        hv = host.numpy()
        for off, a in self.items:
            b = np.frombuffer(a, dtype=np.uint8) if isinstance(a, ctypes.Array) else a.view(np.uint8)
            hv[off:off + b.size] = b
        self.dev.copy_(host, non_blocking=True)


def gt_segments(lab):
    """Run-length ground truth of a frame label vector: (starts, ends inclusive, classes) int32
    (torch_class_label_to_segment_label, utils.py / loss.py:58-84)."""
    lab = np.asarray(lab)
    change = np.ones(len(lab), dtype=bool)
    change[1:] = lab[1:] != lab[:-1]
    st = np.nonzero(change)[0]
    en = np.append(st[1:] - 1, len(lab) - 1)
    return st.astype(np.int32), en.astype(np.int32), lab[st].astype(np.int32)


def class_weights(mc, C1):
    """MatchCriterion.set_label's cweight (C1) and the per-segment weight rule (loss.py:58-84)."""
    cw = np.ones(C1, dtype=np.float32)
    cw[-1] = mc.cfg.Loss.nullw
    if mc._class_weight is not None:
        cw[:C1 - 1] = np.asarray(mc._class_weight[:C1 - 1], dtype=np.float32)
    else:
        for i in mc.bg_ids:
            cw[i] = mc.cfg.Loss.bgw
    return cw


def segment_weights(mc, transcript):
    if mc._class_weight is not None:
        return np.asarray(mc._class_weight, dtype=np.float32)[transcript]
    sw = np.ones(len(transcript), dtype=np.float32)
    for i in mc.bg_ids:
        sw[transcript == i] = mc.cfg.Loss.bgw
    return sw


def supported(net):
    """The fused phase covers FACT / FACT_CLIP without transcripts whose last block has token->frame
    attention (every reference config: the matching reads it).  A batch in which some video's matching
    pairs more than FX_LOSS_MAXK columns makes run() raise TableTooLarge once the matching is known:
    the per-frame predictions (fx_eval_pred) are already enqueued by then (they only read the network's
    outputs and are recomputed by the fallback), but none of the loss launches is; the caller computes
    that batch's losses per video (loss.py's methods)."""
    from .blocks import UpdateBlock, UpdateBlockTDU
    mc = getattr(net, "mcriterion", None)
    if mc is None or net.cfg.FACT.trans or net.cfg.Loss.match not in ("o2o", "o2m", "seq"):
        return False
    return isinstance(net.block_list[-1], (UpdateBlock, UpdateBlockTDU))


def _ptr_rows(t, row0, ld):
    return t.data_ptr() + 4 * row0 * ld


_PENDING = []          # read-backs not resolved yet (resolved at the next forward at the latest)
LAZY_READBACK = os.environ.get("FX_LAZY_READBACK", "1") != "0"   # 0: resolve inside the forward (A/B)
RUN_TIMES = [] if os.environ.get("FX_VLOSS_TIMES") == "1" else None   # diagnostic: host time stamps of run()


def _stamp(name):
    if RUN_TIMES is not None:
        import time
        RUN_TIMES.append((name, time.perf_counter()))


class LazySave(dict):
    """One video's save dict (``pred``, ``loss``) of a step whose host read-back is still in flight:
    every read resolves the read-back first (waiting for the device only if it has not finished).  If
    the read-back carried a kernel failure, every later read re-raises that error.  Pickling / copying
    resolves first and yields a plain dict (the reference's Checkpoint pickles these saves)."""
    __slots__ = ("_pending", "_error")

    def __init__(self, pending):
        super().__init__()
        self._pending = pending
        self._error = None

    def _r(self):
        if self._pending is not None:
            self._pending.resolve()
        if self._error is not None:
            raise self._error

    def __reduce__(self):
        self._r()
        return (dict, (dict(dict.items(self)),))

    def __copy__(self):
        self._r()
        return dict(dict.items(self))

    def __deepcopy__(self, memo):
        import copy
        self._r()
        return copy.deepcopy(dict(dict.items(self)), memo)

    def __getitem__(self, k):
        self._r()
        return dict.__getitem__(self, k)

    def get(self, k, default=None):
        self._r()
        return dict.get(self, k, default)

    def __contains__(self, k):
        self._r()
        return dict.__contains__(self, k)

    def __iter__(self):
        self._r()
        return dict.__iter__(self)

    def __len__(self):
        self._r()
        return dict.__len__(self)

    def keys(self):
        self._r()
        return dict.keys(self)

    def values(self):
        self._r()
        return dict.values(self)

    def items(self):
        self._r()
        return dict.items(self)

    def copy(self):
        self._r()
        return dict(dict.items(self))

    def __eq__(self, other):
        self._r()
        return dict.__eq__(self, other)

    def __repr__(self):
        self._r()
        return dict.__repr__(self)


class PendingReadback:
    """The step's single read-back (predictions, loss floats, kernel status word) as pinned-memory
    copies behind an event; ``resolve`` waits for the event (normally long past), raises a kernel-side
    failure (GRU timeout) and fills the LazySave dicts in place."""

    def __init__(self, ready, check, fill, nvid):
        self.ready, self.check, self.fill = ready, check, fill
        self.saves = [LazySave(self) for _ in range(nvid)]
        self.done = False
        _PENDING.append(self)

    def resolve(self):
        if self.done:
            return
        self.done = True
        if self in _PENDING:
            _PENDING.remove(self)
        for d in self.saves:
            d._pending = None
        self.ready.synchronize()
        try:
            self.check()
        except Exception as e:           # every later read of these saves raises it again
            for d in self.saves:
                d._error = e
            raise
        self.fill(self.saves)


def resolve_pending():
    """Resolve every read-back still in flight (called at the start of each forward), then the
    status copies taken after earlier backward passes (functional.resolve_backward_status)."""
    while _PENDING:
        _PENDING[0].resolve()
    fxf.resolve_backward_status()


class _LossFn(torch.autograd.Function):
    """(out, loss) = fx_loss_terms_fwd(term table): out = [batch loss, per video (loss, fact, contrastive,
    per-block)], loss = out[0] as its own 0-dim output (the step's loss.backward() then enters this node
    directly: no select node, whose backward would zero-fill an nout vector and copy the scalar into it);
    backward writes every input's gradient whole."""

    @staticmethod
    def forward(ctx, plan, *inputs):
        lib = nx.load()
        dev = inputs[0].device
        out = torch.empty(plan["nout"], device=dev, dtype=torch.float32)
        nx.check(lib.fx_loss_terms_fwd(ctypes.addressof(plan["terms_host"]), plan["terms_dev"], plan["nterms"],
                                       plan["coef_dev"], plan["nout"], nx.ptr(out), nx.ptr(plan["ws"]), nx.stream()),
                 "fx_loss_terms_fwd")
        loss = out[0].clone()
        ctx.plan = plan
        ctx.set_materialize_grads(False)
        return out, loss

    @staticmethod
    def backward(ctx, gout, gloss):
        plan = ctx.plan
        lib = nx.load()
        nout = plan["nout"]
        gflat, goff, shapes = plan["grads"]
        if gout is None and gloss is None:
            return (None,) + tuple(None for _ in shapes)
        if gout is None:           # only the batch loss was differentiated: row 0 of the coefficients alone
            gout, nout = gloss.reshape(1).contiguous(), 1
        else:
            gout = gout.contiguous()
            if gloss is not None:
                gout = gout.clone()
                gout[0] += gloss
        nx.check(lib.fx_loss_terms_bwd(ctypes.addressof(plan["terms_host"]), plan["terms_dev"], plan["nterms"],
                                       plan["coef_dev"], nout, nx.ptr(gout), nx.ptr(plan["ws"]), nx.stream()),
                 "fx_loss_terms_bwd")
        rb = plan.get("readback")
        if rb is not None and not rb.done:       # the step's read-back resolves when the backward pass ends
            torch.autograd.Variable._execution_engine.queue_callback(rb.resolve)
        # every input's gradient: its slice of the flat buffer, laid out as the input (contiguous)
        return (None,) + tuple(gflat.as_strided(shp, st, o) for o, (shp, st) in zip(goff, shapes))


def _stage2_labels(net, labs, G):
    """Stage 2's tables that depend on the labels only (EarlyMatch.prepare): the holdout remap and the
    per-video InfoNCE targets (blocks.py:677-747), and the term table's host arrays -- token targets and
    matched-column slots (capacity G[v] >= K), filled after the matching -- in the pack sent with it."""
    from .blocks import FACT_CLIP
    cfg = net.cfg
    nvid = len(labs)
    Q = cfg.FACT.ntoken
    C1 = net.num_classes + 1
    text = getattr(net, "text_embeddings", None) if isinstance(net, FACT_CLIP) else None
    use_clip = text is not None
    con_on = []
    remap = None
    text_seen = text
    if use_clip:
        hold = list(getattr(cfg, "holdout_classes", []) or [])
        if hold:
            n = text.shape[0]
            key = (n, tuple(hold), text.data_ptr(), text._version)
            if getattr(net, "_vloss_text_key", None) != key:
                seen = [i for i in range(n) if i not in set(hold)]
                rm = np.full(n, -1, dtype=np.int64)
                rm[seen] = np.arange(len(seen))
                net._vloss_text = (text[torch.tensor(seen, device=text.device)].contiguous(), rm)
                net._vloss_text_key = key
            text_seen, remap = net._vloss_text
        else:
            text_seen = text.contiguous()
    y_con = []
    for v in range(nvid):
        if not use_clip:
            con_on.append(False)
            y_con.append(None)
            continue
        y = remap[labs[v]] if remap is not None else labs[v]
        con_on.append(bool((y != -1).any()))
        y_con.append(y)
    pk2 = _Pack()
    # per video: token targets (Q) and the matched columns (capacity G[v] >= K), filled after matching
    tgt_arr = [np.full(Q, C1 - 1, dtype=np.int32) for _ in range(nvid)]
    tgt_off = [pk2.array(t, np.int32) for t in tgt_arr]
    tgt_arr = [pk2.items[-nvid + v][1] for v in range(nvid)]     # the buffers pk2 sends
    kcap = [max(int(G[v]), 1) for v in range(nvid)]
    sw_arr, sw_list = [], []
    for v in range(nvid):
        arrs = []
        offs = []
        for dt in (np.int32, np.int32, np.int32, np.float32):
            offs.append(pk2.array(np.zeros(kcap[v], dtype=dt), dt))
            arrs.append(pk2.items[-1][1])
        sw_arr.append(arrs)
        sw_list.append(tuple(offs))
    ycon_off = [pk2.array(y, np.int32) if y is not None and con_on[v] else None for v, y in enumerate(y_con)]
    return dict(use_clip=use_clip, con_on=con_on, y_con=y_con, text_seen=text_seen, pk2=pk2, tgt_off=tgt_off,
                tgt_arr=tgt_arr, kcap=kcap, sw_arr=sw_arr, sw_list=sw_list, ycon_off=ycon_off)


def _contig_strides(shape):
    st, acc = [], 1
    for n in reversed(tuple(shape)):
        st.append(acc)
        acc *= int(n)
    return tuple(reversed(st))


_PINNED = {}


def _pinned(key, shape, dtype):
    """A pinned host buffer reused step after step for one read-back (its previous contents have been read:
    the step's read-back resolves before the next forward's loss phase enqueues the next copy)."""
    t = _PINNED.get(key)
    if t is None or t.shape != torch.Size(shape) or t.dtype != dtype:
        t = _PINNED[key] = torch.empty(shape, dtype=dtype, pin_memory=True)
    return t


class EarlyMatch:
    """Stage 1, called by the LAST block's forward_batch as soon as its token logits and token->frame
    attention exist (before its frame branch and the CLIP head run): ground truth from the host
    labels, one upload, ONE fx_match_cost launch for every video and an asynchronous read-back of
    the costs, so the host's Hungarian overlaps the rest of the forward on the device."""

    def __init__(self, net, hosts):
        self.net, self.hosts = net, hosts
        self.done = False
        self.prepared = False

    def prepare(self, dev):
        """The label-only host work of the loss phase: ground-truth segments, class weights, their upload,
        and the holdout / InfoNCE label tables of stage 2.  The first TDU block runs it while the host
        waits for that block's segment counts (the device is still working through the previous step's
        backward and the first blocks), so none of it is on the host path after the last block, where the
        device would idle behind it; without a TDU block the last block's stage 1 runs it."""
        if self.prepared:
            return
        net = self.net
        C1 = net.num_classes + 1
        gts, labs = [], []
        for lh, ev in self.hosts:
            if ev is not None:
                ev.synchronize()
            lab = lh.numpy() if torch.is_tensor(lh) else np.asarray(lh)
            labs.append(lab)
            gts.append(gt_segments(lab))
        G = [len(g[0]) for g in gts]
        pk = _Pack()
        gt_off = [(pk.array(g[0], np.int32), pk.array(g[1], np.int32), pk.array(g[2], np.int32)) for g in gts]
        lab_off = [pk.array(lab, np.int32) for lab in labs]
        cw = class_weights(net.mcriterion, C1)
        cw_off = pk.array(cw, np.float32)
        base = pk.alloc(dev)
        pk.send()
        self.__dict__.update(labs=labs, gts=gts, G=G, Gmax=max(G), gt_off=gt_off, lab_off=lab_off, cw=cw,
                             cw_off=cw_off, pk=pk, base=base)
        self.stage2 = _stage2_labels(net, labs, G)
        self.prepared = True

    def __call__(self, vb, a_cl, a2f_at, seg=None):
        net, cfg = self.net, self.net.cfg
        lib = nx.load()
        nvid, Q, fo = vb.nvid, vb.Q, vb.f_off
        C1 = net.num_classes + 1
        dev = a_cl.device
        self.prepare(dev)
        G, Gmax, gt_off, base = self.G, self.Gmax, self.gt_off, self.base
        pkv = _Pack()
        va_off, va = pkv.structs(nx.VideoAttn, nvid)
        vbase = pkv.alloc(dev)
        for v in range(nvid):
            a = va[v]
            a.Q, a.C1, a.T, a.G = Q, C1, vb.Ts[v], G[v]
            a.clogit, a.ldc = _ptr_rows(a_cl, v * Q, C1), C1
            if seg is not None:
                s_off, local = seg
                a.attn, a.lda = a2f_at.data_ptr() + 4 * Q * s_off[v], Q
                a.seg_id = local[v][0].data_ptr()
            else:
                a.attn, a.lda = a2f_at.data_ptr() + 4 * Q * fo[v], Q
            a.gs, a.ge, a.gl = (base + o for o in gt_off[v])
            a.pred_off = fo[v]
        pkv.send()
        self.cost_host = None
        if cfg.Loss.match != "seq":
            cost = torch.empty(nvid * Q * Gmax, dtype=torch.float32, device=dev)
            nx.check(lib.fx_match_cost(ctypes.addressof(va), vbase + va_off, nvid, float(cfg.Loss.pc),
                                       float(cfg.Loss.a2fc), Gmax, nx.ptr(cost), nx.stream()), "fx_match_cost")
            self.cost_host = _pinned("cost", cost.shape, torch.float32)
            self.cost_host.copy_(cost, non_blocking=True)
            self.cost_ready = torch.cuda.Event()
            self.cost_ready.record()
            self.cost_dev = cost
        self.pkv = pkv
        self.done = True

    def matches(self, Q):
        """Hungarian / one-to-many / sequential matching per video (loss.py:108-193) on the host."""
        kind = self.net.cfg.Loss.match
        cost = None
        if self.cost_host is not None:
            self.cost_ready.synchronize()
            cost = self.cost_host.numpy().reshape(len(self.G), Q, self.Gmax)
        out = []
        for v, Gv in enumerate(self.G):
            if kind == "seq":
                assert Q >= Gv, (Q, Gv)
                ai = si = np.arange(Gv)
            else:
                c = cost[v, :, :Gv].astype(np.float64)
                if not np.isfinite(c).all():
                    # costs from a step whose kernels reported a failure (e.g. a BiGRU timeout): raise that
                    # failure (the status word is final: the costs' event has completed) rather than the
                    # matching's own error on the garbage it produced
                    st = fxf.device_status(self.cost_dev.device)
                    fxf.status_raise(int(st[0].item()), self.cost_dev.device)
                ai, si = linear_sum_assignment(c) if kind == "o2o" else one_to_many_match(c, self.gts[v][2])
            out.append((np.asarray(ai, dtype=np.int64), np.asarray(si, dtype=np.int64)))
        return out


class TableTooLarge(Exception):
    """A video of the batch pairs more matched token/segment columns than the fused term table holds
    (FX_LOSS_MAXK): the caller runs that batch's losses on the per-video path instead."""


def run(net, vb, compute_loss, early=None):
    """Predictions (and with compute_loss the batch loss + per-video loss values) of the lockstep
    batch whose block outputs forward_batch left in ``blk._bt``; ``early`` is the EarlyMatch the last
    block already ran.  Returns what _forward_videos returns: save_list, or (loss, save_list)."""
    from .blocks import FACT_CLIP, InputBlock, UpdateBlockTDU
    lib = nx.load()
    cfg = net.cfg
    blocks = list(net.block_list)
    last = blocks[-1]._bt
    nvid, Q, Ts, fo = vb.nvid, vb.Q, vb.Ts, vb.f_off
    C = net.num_classes
    C1 = C + 1
    dev = last["f_cl"].device
    mc = net.mcriterion
    clip = isinstance(net, FACT_CLIP)
    text = getattr(net, "text_embeddings", None) if clip else None
    proj = getattr(net, "_proj", None) if clip else None
    use_clip = text is not None and proj is not None
    flog = fxf.matmul_nt(proj.detach(), text, alpha=1.0 / cfg.CLIP.temp) if use_clip else last["f_cl"]

    def eval_structs(pk):
        off, va = pk.structs(nx.VideoAttn, nvid)
        for v in range(nvid):
            a = va[v]
            a.Q, a.C1, a.T = Q, C1, Ts[v]
            a.clogit, a.ldc = _ptr_rows(last["a_cl"], v * Q, C1), C1
            if "S" in last:
                a.attn, a.lda = last["a2f_at"].data_ptr() + 4 * Q * last["s_off"][v], Q
                a.seg_id = last["local"][v][0].data_ptr()
            else:
                a.attn, a.lda = last["a2f_at"].data_ptr() + 4 * Q * fo[v], Q
            a.flogit, a.ldf = _ptr_rows(flog, fo[v], C), C
            a.pred_off = fo[v]
        return off, va

    _stamp("pred")
    pred = torch.empty(fo[-1], dtype=torch.int32, device=dev)
    if not compute_loss:
        pk = _Pack()
        va_off, va = eval_structs(pk)
        base = pk.alloc(dev)
        pk.send()
        nx.check(lib.fx_eval_pred(ctypes.addressof(va), base + va_off, nvid, float(cfg.FACT.mwt), nx.ptr(pred),
                                  nx.stream()), "fx_eval_pred")
        host = torch.cat([pred, fxf.device_status(dev)[:1]]).cpu().numpy()
        fxf.status_raise(int(host[-1]), dev)
        return [{"pred": host[fo[v]:fo[v + 1]].astype(np.int64)} for v in range(nvid)]

    assert early is not None and early.done, "the last block did not run the early matching stage"
    # Everything that does not depend on the matching is built first, while the device still works
    # through the end of the forward: the term table with room for the matched columns (K <= G
    # segments of the video), the structs, the scratch layout, and the prediction launch.  Only then
    # does the host wait for the match costs; after the Hungarian it fills the token targets and the
    # matched columns, sets K and the token-CE normaliser, sends the table and launches the loss.
    labs, gts, G, gt_off, lab_off = early.labs, early.gts, early.G, early.gt_off, early.lab_off
    cw, cw_off, base = early.cw, early.cw_off, early.base

    # ------------------------------------------------------------------ stage 2: the term table
    sw_coef = float(cfg.Loss.sw)
    nb = len(blocks)
    if not early.prepared:
        early.prepare(dev)
    st2 = early.stage2
    con_on, y_con, text_seen = st2["con_on"], st2["y_con"], st2["text_seen"]
    pk2, tgt_off, tgt_arr, kcap = st2["pk2"], st2["tgt_off"], st2["tgt_arr"], st2["kcap"]
    sw_arr, sw_list, ycon_off = st2["sw_arr"], st2["sw_list"], st2["ycon_off"]
    if use_clip != st2["use_clip"]:
        raise RuntimeError("vloss: the CLIP head ran differently from the prepared label tables")

    _stamp("con")
    # the predictions (no matching needed): own small table, launched before the wait
    pke = _Pack()
    va_off, va = eval_structs(pke)
    pke.alloc(dev)
    pke.send()
    nx.check(lib.fx_eval_pred(ctypes.addressof(va), pke.base + va_off, nvid, float(cfg.FACT.mwt), nx.ptr(pred),
                              nx.stream()), "fx_eval_pred")

    _stamp("eval_pred")
    _stamp("pk2_arrays")
    # every differentiated input of the term table, its gradient a view of ONE flat allocation
    inputs, gidx = [], {}

    def want(t):
        if id(t) not in gidx:
            gidx[id(t)] = len(inputs)
            inputs.append(t)
    for blk in blocks:
        bt = blk._bt
        for key in ("f_cl", "a_cl", "seg_cl", "f2a_lg", "a2f_lg"):
            if key in bt and not (key.endswith("_lg") and isinstance(blk, InputBlock)):
                want(bt[key])
    if any(con_on):
        want(proj)
    sizes = [(t.numel() + 63) & ~63 for t in inputs]      # 256-byte aligned slices
    gflat = torch.empty(sum(sizes), device=dev, dtype=torch.float32)
    goff, o_ = [], 0
    for n_ in sizes:
        goff.append(o_)
        o_ += n_
    gb = gflat.data_ptr()

    class _G:       # an input's gradient slice by address only; the tensors are made in the backward
        __slots__ = ("p",)

        def __init__(self, p):
            self.p = p

        def data_ptr(self):
            return self.p

    def grad_of(t):
        return _G(gb + 4 * goff[gidx[id(t)]])

    # The term table in ONE pass straight into the ABI structs (their count is known from the block types:
    # frame CE + token CE per block and video, + the segment CE for a TDU block, + the f2a / a2f cross-
    # attention CE for an update block, + one InfoNCE term per video with a contrastive target); the
    # pointers into the two packs resolve at once (both are allocated before the structs are filled)
    nper = [2 if isinstance(blk, InputBlock) else 5 if isinstance(blk, UpdateBlockTDU) else 4 for blk in blocks]
    nterms = nvid * sum(nper) + sum(1 for c in con_on if c)
    per = 3 + nb
    nout = 1 + nvid * per
    coef_off = pk2.array(np.zeros((nout, nterms), dtype=np.float32), np.float32)
    coef = pk2.items[-1][1].reshape(nout, nterms)          # (the buffer pk2 sends)
    t_off, terms = pk2.structs(nx.LossTerm, nterms)
    base2 = pk2.alloc(dev)
    fw, cwt = float(getattr(cfg.CLIP, "fact_loss_weight", 1.0)), float(getattr(cfg.CLIP, "contrastive_weight", 0.0))
    tok_terms, attn_terms = [], []     # (term index, video): fields set after the matching
    slots = []                         # scratch sizes (lse, lse2, colz) per term
    # coefficient matrix: out = [batch loss, per video (loss, fact, contrastive, block values...)]
    lw_blk = [fw / nb if con_on[v] else 1.0 / nb for v in range(nvid)]
    nxt = [0]

    def term(k, v, kind, R, Cc, x, sr, sc, dx, dsr, dsc, c_ce, c_sm, n_lse, n_lse2, n_colz):
        i = nxt[0]
        nxt[0] = i + 1
        t = terms[i]
        t.slot, t.kind, t.R, t.C, t.x, t.sr, t.sc = i, kind, R, Cc, x, sr, sc
        t.dx, t.dsr, t.dsc, t.c_ce, t.c_sm = dx, dsr, dsc, c_ce, c_sm
        slots.append((n_lse, n_lse2, n_colz))
        o = 1 + v * per
        if k >= 0:
            coef[o + 3 + k, i] = 1.0
            coef[o + 1, i] = 1.0 / nb
            lw = lw_blk[v]
        else:
            coef[o + 2, i] = 1.0
            lw = cwt
        coef[o, i] = lw
        coef[0, i] = lw / nvid
        return i, t

    cw_p = base + cw_off
    for k, blk in enumerate(blocks):
        bt = blk._bt
        is_tdu = isinstance(blk, UpdateBlockTDU)
        f_cl, a_cl = bt["f_cl"], bt["a_cl"]
        pf, pa = f_cl.data_ptr(), a_cl.data_ptr()
        gf, ga = grad_of(f_cl).data_ptr(), grad_of(a_cl).data_ptr()
        fce = 0.5 if is_tdu else 1.0
        if not isinstance(blk, InputBlock):
            f2a, a2f = bt["f2a_lg"], bt["a2f_lg"]
            pfa, paf = f2a.data_ptr(), a2f.data_ptr()
            gfa, gaf = grad_of(f2a).data_ptr(), grad_of(a2f).data_ptr()
            if is_tdu:
                seg_cl = bt["seg_cl"]
                psg, gsg = seg_cl.data_ptr(), grad_of(seg_cl).data_ptr()
        for v in range(nvid):
            gs, ge, gl = gt_off[v]
            T = Ts[v]
            # frame CE (+ smooth) on the block's frame logits
            _, t = term(k, v, nx.TERM_CLASS, T, C, pf + 4 * fo[v] * C, C, 1, gf + 4 * fo[v] * C, C, 1, fce / T,
                        (sw_coef / ((T - 1) * C) if sw_coef and T > 1 else 0.0), T, 0, 0)
            t.y, t.w = base + lab_off[v], cw_p
            # token CE (c_ce = 1 / the targets' class-weight sum, after the matching)
            i, t = term(k, v, nx.TERM_CLASS, Q, C1, pa + 4 * v * Q * C1, C1, 1, ga + 4 * v * Q * C1, C1, 1, 0.0, 0.0,
                        Q, 0, 0)
            t.y, t.w = base2 + tgt_off[v], cw_p
            tok_terms.append((i, v))
            if isinstance(blk, InputBlock):
                continue
            ka_o, kgs_o, kge_o, ksw_o = sw_list[v]
            Kc = kcap[v]
            if is_tdu:
                Sv, s0 = bt["S"][v], bt["s_off"][v]
                rs, re = bt["local"][v][1].data_ptr(), bt["local"][v][2].data_ptr()
                _, t = term(k, v, nx.TERM_CLASS, Sv, C, psg + 4 * s0 * C, C, 1, gsg + 4 * s0 * C, C, 1, 0.5 / Sv, 0.0,
                            Sv, 0, 0)
                t.rs, t.re, t.gs, t.ge, t.gl, t.G, t.w = rs, re, base + gs, base + ge, base + gl, G[v], cw_p
                R, off, c_xe, c_sm = Sv, Q * s0, 1.0 / Sv, 0.0
            else:
                rs = re = None
                R, off = T, Q * fo[v]
                c_xe, c_sm = 1.0 / T, (sw_coef / ((T - 1) * Q) if sw_coef and T > 1 else 0.0)
            # f2a logits (Q, R) read as (R, Q): log_softmax over rows per matched column (dim=1)
            for x, dx, sr, sc, axis in ((pfa, gfa, 1, R, 0), (paf, gaf, Q, 1, 1)):
                i, t = term(k, v, nx.TERM_ATTN, R, Q, x + 4 * off, sr, sc, dx + 4 * off, sr, sc, c_xe, c_sm,
                            R, R + Kc, Kc)
                t.rs, t.re, t.axis = rs, re, axis
                t.ka, t.kgs, t.kge, t.ksw = base2 + ka_o, base2 + kgs_o, base2 + kge_o, base2 + ksw_o
                attn_terms.append((i, v))
    _stamp("specs")
    sims = None
    if any(con_on):
        Cs = text_seen.shape[0]
        Dc = text_seen.shape[1]
        sims = torch.empty(2, fo[-1], Cs, device=dev)
        ncolz = ((Cs + 4) & ~3) + 4 * nx.LOSS_NB * Cs
        gp = grad_of(proj)
        if not all(con_on):     # (videos without a contrastive target leave their projection rows at zero)
            i_ = gidx[id(proj)]
            gflat.narrow(0, goff[i_], proj.numel()).zero_()
        p0, p1, pe, pg = sims[0].data_ptr(), sims[1].data_ptr(), proj.data_ptr(), gp.data_ptr()
        inv_temp = 1.0 / float(cfg.CLIP.temp)
        for v in range(nvid):
            if not con_on[v]:
                continue
            T = Ts[v]
            _, t = term(-1, v, nx.TERM_INFONCE, T, Cs, p0 + 4 * fo[v] * Cs, Cs, 1, p1 + 4 * fo[v] * Cs, Cs, 1, 0.5, 0.0,
                        T, Cs, ncolz)
            t.y, t.emb, t.ld_emb, t.text, t.D = base2 + ycon_off[v], pe + 4 * fo[v] * Dc, Dc, text_seen.data_ptr(), Dc
            t.inv_temp, t.demb, t.ld_demb = inv_temp, pg + 4 * fo[v] * Dc, Dc
    assert nxt[0] == nterms, (nxt[0], nterms)
    _stamp("infonce")
    _stamp("coef")
    # per-term scratch: lse, lse2, colz slots (16-byte aligned)
    offs, sc_ = [], 0
    for sz in slots:
        o3 = []
        for n in sz:
            o3.append(sc_)
            sc_ += (max(n, 1) + 3) & ~3
        offs.append(o3)
    scr = torch.empty(max(sc_, 1), device=dev, dtype=torch.float32)
    sbase = scr.data_ptr()
    for i, o3 in enumerate(offs):
        t = terms[i]
        t.lse, t.lse2, t.colz = sbase + 4 * o3[0], sbase + 4 * o3[1], sbase + 4 * o3[2]
    _stamp("structs")
    ws = torch.empty(max(lib.fx_loss_terms_workspace_floats(nterms), 1), device=dev, dtype=torch.float32)

    # ------------------------------------------------------------------ the matching (waits for the costs)
    matches = early.matches(Q)
    _stamp("matches")
    big = [v for v, (ai, _) in enumerate(matches) if len(ai) > nx.LOSS_MAXK]
    if big:      # e.g. o2m matching (every ground-truth segment paired, loss.py:155-193) past 512 segments
        raise TableTooLarge(big)
    ksum = []
    for v in range(nvid):
        ai, si = matches[v]
        K = len(ai)
        if K > kcap[v]:
            raise RuntimeError(f"video {v}: {K} matched columns > {kcap[v]} ground-truth segments")
        tgt = tgt_arr[v]
        tgt[ai] = gts[v][2][si]
        ksum.append(float(cw[tgt].sum()))
        swn = segment_weights(mc, gts[v][2])
        if len(swn) not in (K, 1):
            raise RuntimeError(f"cross_attn_loss: {K} matched columns vs {len(swn)} segment weights")
        ka, kgs, kge, ksw = sw_arr[v]
        ka[:K] = ai
        kgs[:K] = gts[v][0][si]
        kge[:K] = gts[v][1][si]
        ksw[:K] = swn if len(swn) == K else swn[0]
    for i, v in tok_terms:
        terms[i].c_ce = 1.0 / ksum[v]
    for i, v in attn_terms:
        terms[i].K = len(matches[v][0])
    _stamp("fill")
    pk2.send()
    _stamp("send")
    plan = dict(terms_host=terms, terms_dev=base2 + t_off, nterms=nterms, coef_dev=base2 + coef_off, nout=nout,
                ws=ws, grads=(gflat, goff, [(t.shape, _contig_strides(t.shape)) for t in inputs]),
                keep=(early, pk2, pke, scr, sims, flog, text_seen))
    out, loss = _LossFn.apply(plan, *inputs)

    _stamp("send_lossfn")
    # the reference's side channels: last video's per-block losses, fact / contrastive terms
    # (blocks.py:905-910: a video without a contrastive term reports the attributes an earlier
    # video -- or an earlier call -- left behind, as the reference's hasattr checks do)
    prev = None
    if not all(con_on) and hasattr(net, "fact_loss") and hasattr(net, "contrastive_loss"):
        # read at resolve time: float() of a device value here would drain the stream (the loss
        # kernels just issued included) before the backward is issued
        prev = (net.fact_loss, net.contrastive_loss)
    o = 1 + (nvid - 1) * per
    from .blocks import _OutRef
    d = net.__dict__              # lazily indexed (blocks._lazy_out_attr), no nn.Module.__setattr__ walk
    d["_lo_loss_list"] = _OutRef(out, list(range(o + 3, o + 3 + nb)))
    for v in range(nvid):
        if con_on[v]:
            o = 1 + v * per
            d["_lo_fact_loss"], d["_lo_contrastive_loss"] = _OutRef(out, o + 1), _OutRef(out, o + 2)
    # ONE device->host read-back for the predictions and every loss value, enqueued here and resolved
    # later: at the end of the backward pass (autograd callback queued by _LossFn.backward), at the first
    # read of a save entry, or at the next forward -- whichever comes first -- so loss.backward() is
    # issued while the device still finishes the forward instead of after a drain
    _stamp("side")
    out_h = _pinned("out", out.shape, torch.float32)
    pred_h = _pinned("pred", pred.shape, torch.int32)
    st_h = _pinned("status", (1,), torch.int32)
    out_h.copy_(out.detach(), non_blocking=True)
    pred_h.copy_(pred, non_blocking=True)
    st_h.copy_(fxf.device_status(dev)[:1], non_blocking=True)   # kernel-side failures (GRU timeout)
    ready = torch.cuda.Event()
    ready.record()

    _stamp("readback")
    def fill(saves):
        vals = out_h.tolist()
        ph = pred_h.numpy()
        prev_ = None if prev is None else tuple(float(x) for x in prev)
        for v in range(nvid):
            o = 1 + v * per
            d = {"loss": vals[o]}
            if con_on[v]:
                prev_ = (vals[o + 1], vals[o + 2])
            if prev_ is not None:
                d["fact_loss"], d["contrastive_loss"] = prev_
            saves[v]["pred"] = ph[fo[v]:fo[v + 1]].astype(np.int64)
            saves[v]["loss"] = d
    pending = PendingReadback(ready, lambda: fxf.status_raise(int(st_h[0]), dev), fill, nvid)
    plan["readback"] = pending
    if not LAZY_READBACK:
        pending.resolve()
    return loss, pending.saves
