"""Autograd functions over the libfactmx C ABI.

Every function here launches hand-written HIP kernels through ``native`` on
PyTorch's current stream; tensors are fp32 row-major (rows, channels).  There
is no eager/CPU fallback: a missing library raises FactmxNativeError.

Gradient convention: the kernels ACCUMULATE weight and bias gradients (+=)
straight into ``param.grad`` of leaf parameters (allocating zeros on first use,
exactly what autograd's AccumulateGrad would do) and the backward returns
``None`` for them.  With ``factmx.dp.FlatGradReducer`` those ``.grad`` tensors
are views into the all-reduce buckets, so no per-parameter add, fill or copy
kernel is launched.  Non-leaf weights get a fresh buffer that is returned to
autograd as usual.
"""
import ctypes
import os

import torch

from . import native as nx

_f32 = torch.float32


def _empty(*shape, device):
    return torch.empty(*shape, device=device, dtype=_f32)


def _ws(n, device):
    return torch.empty(max(int(n), 1), device=device, dtype=_f32)


# ---------------------------------------------------------------------------
# The library's side stream: weight-gradient GEMMs (MS-TCN backward) run there and are joined
# only when the gradients are needed (end of the backward pass, or before a DP bucket all-reduce),
# so they overlap the following blocks' latency-bound token-side backward.
# ---------------------------------------------------------------------------
DEFER_SIDE = True
_side = None
_join_pending = False


def side_stream():
    """torch view of fx_side_stream() (None when the library has none)."""
    global _side
    if _side is None:
        h = nx.load().fx_side_stream()
        _side = torch.cuda.ExternalStream(h, device=torch.cuda.current_device()) if h else False
    return _side or None


def side_join():
    """Make the current stream wait for the work deferred to the side stream (no-op when none)."""
    global _join_pending
    if _join_pending:
        _join_pending = False
        _check(nx.load().fx_side_join(nx.stream()), "fx_side_join")


def _defer_to_side(*tensors):
    """The side stream still reads `tensors`: keep the allocator from reusing them early, and join
    at the end of the running backward pass."""
    global _join_pending
    s = side_stream()
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    if not _join_pending:
        _join_pending = True
        torch.autograd.Variable._execution_engine.queue_callback(side_join)


def _may_defer(tg):
    """Weight gradients may stay on the side stream past this backward call only when every target
    is a leaf's .grad (joined at the end of the backward pass).  A non-leaf parameter's gradient is a
    fresh buffer handed back to autograd, which reads it on the main stream right away: then the
    entry point joins its side work before returning (side_defer = 0)."""
    return DEFER_SIDE and side_stream() is not None and all(t[1] is None for t in tg)


class gemm_precision:
    """Context manager (or plain call) for the GEMM arithmetic of work enqueued on the CURRENT torch
    stream: "fp32" (default, the parity path) or "bf16" (FX_PREC_BF16: frame-level forward /
    input-gradient products on bf16 MFMA with fp32 accumulation and storage; a performance mode whose
    deviation bench.py reports).  Per stream (fx_set_stream_precision): other streams and threads keep
    their own setting."""

    def __init__(self, mode, stream=None):
        modes = PRECISIONS
        if mode not in modes:
            raise ValueError(f"gemm precision {mode!r}: one of {sorted(modes)}")
        lib = nx.load()
        self._stream = nx.stream() if stream is None else stream.cuda_stream
        self._prev = lib.fx_stream_precision_explicit(self._stream)   # PREC_DEFAULT when never set
        nx.check(lib.fx_set_stream_precision(self._stream, modes[mode]), "fx_set_stream_precision")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        nx.check(nx.load().fx_set_stream_precision(self._stream, self._prev), "fx_set_stream_precision")
        return False


PRECISIONS = {"fp32": nx.PREC_F32, "bf16": nx.PREC_BF16, "fp32s": nx.PREC_F32S, "fp32s2": nx.PREC_F32S2}


def set_default_precision(mode):
    """Library-wide GEMM arithmetic of streams without their own setting (fx_set_default_precision):
    "fp32s" (fp32 on the bf16 matrix cores by a 3-piece split), "fp32" (f32 MFMA), ..."""
    if mode not in PRECISIONS:
        raise ValueError(f"gemm precision {mode!r}: one of {sorted(PRECISIONS)}")
    nx.check(nx.load().fx_set_default_precision(PRECISIONS[mode]), "fx_set_default_precision")


def default_precision():
    inv = {v: k for k, v in PRECISIONS.items()}
    return inv[nx.load().fx_get_default_precision()]


def dropout_seed():
    """Seed of one training dropout site, drawn from torch's default CPU generator (so
    torch.manual_seed fixes the masks, as it fixes nn.Dropout's); the kernels derive every mask
    element from it by a counter-based hash and regenerate it in backward."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def dropout(x, p, seed):
    """fx_dropout on a (rows, cols) tensor: x * keep / (1 - p) with the kernels' mask."""
    lib = nx.load()
    x2 = _2d(x).contiguous()
    y = torch.empty_like(x2)
    rows, cols = x2.shape
    _check(lib.fx_dropout(nx.ptr(x2), cols, rows, cols, cols, 0, float(p), int(seed), nx.ptr(y), cols, nx.stream()),
           "fx_dropout")
    return y


def _2d(t):
    """(N, 1, C) or (N, C) -> (N, C) view with unit column stride."""
    if t.dim() == 3:
        assert t.shape[1] == 1, t.shape
        t = t.squeeze(1)          # a view: its backward is a view too (t[:, 0] would zero-fill + copy)
    if t.stride(-1) != 1:
        t = t.contiguous()
    return t


def _w2d(w):
    return w.reshape(w.shape[0], -1) if w.dim() == 3 else w


def _check(status, what):
    if status != 0:
        nx.check(status, what)


def grad_target(p, needed=True):
    """(buffer the kernel accumulates into, value to return to autograd)."""
    if p is None or not needed:
        return None, None
    if p.is_leaf:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
        return p.grad, None
    buf = torch.zeros_like(p)
    return buf, buf


class PosGradSink:
    """One gradient buffer for a position table that several fused ops read (the action queries
    repeated per video: every block's decoder query_pos and both cross-attention maps, blocks.py
    _forward_batch).  Each op's backward ACCUMULATES its position gradient into ``buf`` (the first one
    writes it) and returns None for it; ``PosSinkFn``'s backward -- which autograd runs only after every
    op reading its output has run its own -- hands the sum on.  Without it the engine adds the per-op
    position gradients pairwise (one add launch per extra reader, ~10 per headline step)."""

    def __init__(self):
        self.buf = None

    def target(self, shape, dev):
        """(buffer, accumulate flag) for one reader's position gradient."""
        if self.buf is None:
            self.buf = _empty(*shape, device=dev)
            return self.buf, 0
        assert tuple(self.buf.shape) == tuple(shape), (self.buf.shape, shape)
        return self.buf, 1


class PosSinkFn(torch.autograd.Function):
    """Identity on a position table whose readers accumulate into one PosGradSink (see there)."""

    @staticmethod
    def forward(ctx, pos, sink):
        ctx.sink = sink
        ctx.set_materialize_grads(False)
        return pos.view_as(pos)

    @staticmethod
    def backward(ctx, g):
        buf, ctx.sink.buf = ctx.sink.buf, None
        if buf is None:
            return g, None
        if g is not None:        # readers outside the fused ops (plain torch) returned theirs
            buf.add_(g)
        return buf, None


# FX_POS_SINK=0: every reader returns its own position gradient (autograd adds them; A/B knob)
POS_SINK = int(os.environ.get("FX_POS_SINK", "1"))


def pos_sink(pos):
    """``pos`` wrapped so that the fused ops reading it share one gradient buffer (PosGradSink);
    ``pos`` itself when it needs no gradient."""
    if pos is None or not (POS_SINK and pos.requires_grad and torch.is_grad_enabled()):
        return pos
    sink = PosGradSink()
    out = PosSinkFn.apply(pos, sink)
    out._fx_pos_sink = sink
    return out


def _sink_of(t):
    return None if t is None else getattr(t, "_fx_pos_sink", None)


# ---------------------------------------------------------------------------
# raw launch helpers (no autograd)
# ---------------------------------------------------------------------------

def lin_fwd(x, w, b, relu=0, out=None):
    lib = nx.load()
    w2 = _w2d(w)
    M, K = x.shape
    N = w2.shape[0]
    y = out if out is not None else _empty(M, N, device=x.device)
    _check(lib.fx_linear_fwd(nx.ptr(x), nx.ld(x), None, 0, 0, M, K, nx.ptr(w2), nx.ld(w2), nx.ptr(b),
                             nx.ptr(y), nx.ld(y), N, int(relu), nx.stream()), "fx_linear_fwd")
    return y


def lin_bwd(dy, x, w, need_dx=True, dw=None, db=None, relu_out=None, dx_out=None, acc_dx=False):
    """dx = dy.w (returned / written to dx_out); dw += dy^T x and db += colsum(dy) when given."""
    lib = nx.load()
    w2 = _w2d(w)
    M, K = x.shape
    N = w2.shape[0]
    dev = dy.device
    dx = dx_out if dx_out is not None else (_empty(M, K, device=dev) if need_dx else None)
    dw2 = None if dw is None else (dw.reshape(dw.shape[0], -1) if dw.dim() == 3 else dw)
    ws = _ws(lib.fx_linear_bwd_workspace_floats(M, K, N), dev)
    _check(lib.fx_linear_bwd(nx.ptr(dy), nx.ld(dy), nx.ptr(x), nx.ld(x), nx.ptr(w2), nx.ld(w2),
                             nx.ptr(relu_out), nx.ld(relu_out), M, K, N, nx.ptr(dx), nx.ld(dx),
                             nx.ptr(dw2), nx.ld(dw2), nx.ptr(db), int(acc_dx), 1, nx.ptr(ws), nx.stream()),
           "fx_linear_bwd")
    return dx


# ---------------------------------------------------------------------------
# Linear / Conv1d(k=1)
# ---------------------------------------------------------------------------

class LinearFn(torch.autograd.Function):
    """nn.Linear / Conv1d(k=1) on (rows, K): basic.py:139,177,182; blocks.py:154,158,402,414."""

    @staticmethod
    def forward(ctx, x, w, b, relu):
        y = lin_fwd(x, w, b, relu)
        ctx.relu = relu
        ctx.has_b = b is not None
        ctx.save_for_backward(x, w, b, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, y = ctx.saved_tensors
        nd = ctx.needs_input_grad
        dwb, dw_ret = grad_target(w, nd[1])
        dbb, db_ret = grad_target(b, nd[2] and ctx.has_b)
        dx = lin_bwd(dy.contiguous(), x, w, nd[0], dwb, dbb, relu_out=y if ctx.relu else None)
        return dx, dw_ret, db_ret, None


def linear(x, w, b, relu=False):
    return LinearFn.apply(_2d(x), w, b, int(relu))


class LinearPadKFn(torch.autograd.Function):
    """nn.Linear for an in-feature count K that is not a multiple of the GEMM's 64-deep stage, on an
    input that is a column slice of a wider row-major tensor (FeatureProjection's x[:, :H-C],
    blocks.py:168-170): the GEMMs run over Kp = ceil64(K) against a zero-padded copy of W, so every
    operand is 16-B vector-loadable (the extra input columns meet zero weights).  Same values as
    the unpadded product (the padded terms are exact zeros)."""

    @staticmethod
    def forward(ctx, x, w, b, Kp):
        M, K = x.shape
        N = w.shape[0]
        wp = torch.nn.functional.pad(w.detach(), (0, Kp - K))
        y = _empty(M, N, device=x.device)
        gemm(M, N, Kp, _rows_operand(x), _rows_operand(wp), y, N, bias=b)
        ctx.save_for_backward(x, w, b, wp)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b, wp = ctx.saved_tensors
        nd = ctx.needs_input_grad
        dy = dy.contiguous()
        M, K = x.shape
        N = w.shape[0]
        dx = None
        if nd[0]:
            dx = _empty(M, K, device=dy.device)
            o = nx.Operand()
            o.ptr, o.ld, o.trans, o.conv_dir = nx.ptr(wp), wp.shape[1], 1, 1
            gemm(M, K, N, _rows_operand(dy), o, dx, K)
        dwb, dw_ret = grad_target(w, nd[1])
        dbb, db_ret = grad_target(b, nd[2])
        if dwb is not None or dbb is not None:
            lin_bwd(dy, x, w, False, dwb, dbb)
        return dx, dw_ret, db_ret, None


def linear_any_k(x, w, b):
    """linear() that pads K to the 64-deep GEMM stage when x has the room to be read that wide."""
    x2 = _2d(x)
    M, K = x2.shape
    Kp = (K + 63) // 64 * 64
    if K % 64 == 0 or x2.stride(1) != 1 or x2.stride(0) < Kp or x2.stride(0) % 4 or x2.data_ptr() % 16:
        return LinearFn.apply(x2, w, b, 0)
    last = x2.storage_offset() + (M - 1) * x2.stride(0) + Kp
    if last > x2.untyped_storage().nbytes() // x2.element_size():
        return LinearFn.apply(x2, w, b, 0)
    return LinearPadKFn.apply(x2, w, b, Kp)


# ---------------------------------------------------------------------------
# LayerNorm (+ fused residual, + fused ReLU)
# ---------------------------------------------------------------------------

class LayerNormFn(torch.autograd.Function):
    """post-norm ``LN(x + r)`` (basic.py:444-450, 504-522; blocks.py:155-156 with ReLU)."""

    @staticmethod
    def forward(ctx, x, r, w, b, eps, relu):
        lib = nx.load()
        rows, cols = x.shape
        y = _empty(rows, cols, device=x.device)
        xhat = _empty(rows, cols, device=x.device)
        rstd = _empty(rows, device=x.device)
        _check(lib.fx_layernorm_fwd(nx.ptr(x), nx.ld(x), nx.ptr(r), nx.ld(r), nx.ptr(w), nx.ptr(b), float(eps),
                                    rows, cols, int(relu), nx.ptr(y), cols, nx.ptr(xhat), cols, nx.ptr(rstd),
                                    nx.stream()), "fx_layernorm_fwd")
        ctx.relu = relu
        ctx.has_r = r is not None
        ctx.save_for_backward(y, xhat, rstd, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = nx.load()
        y, xhat, rstd, w, b = ctx.saved_tensors
        nd = ctx.needs_input_grad
        dy = dy.contiguous()
        rows, cols = y.shape
        dev = dy.device
        dx = _empty(rows, cols, device=dev)
        dwb, dw_ret = grad_target(w, nd[2])
        dbb, db_ret = grad_target(b, nd[3])
        ws = _ws(lib.fx_layernorm_bwd_workspace_floats(rows, cols), dev)
        _check(lib.fx_layernorm_bwd(nx.ptr(dy), cols, nx.ptr(y), cols, nx.ptr(xhat), cols, nx.ptr(w), nx.ptr(rstd),
                                    rows, cols, int(ctx.relu), nx.ptr(dx), cols, nx.ptr(dwb), nx.ptr(dbb), nx.ptr(ws),
                                    nx.stream()), "fx_layernorm_bwd")
        return dx, (dx if ctx.has_r else None), dw_ret, db_ret, None, None


def layer_norm(x, w, b, eps=1e-5, residual=None, relu=False):
    return LayerNormFn.apply(_2d(x), None if residual is None else _2d(residual), w, b, eps, int(relu))


# ---------------------------------------------------------------------------
# process_feature (class-logit softmax tail)
# ---------------------------------------------------------------------------

class ProcessFeatureFn(torch.autograd.Function):
    """``Block.process_feature`` (blocks.py:195-202): out = [x[:, :-n], softmax(x[:, -n:])] and the
    class logits x[:, -n:] as a second output, so their gradient (from the losses) enters the
    backward kernel directly instead of through a zero-filled slice gradient plus an add."""

    @staticmethod
    def forward(ctx, x, n):
        lib = nx.load()
        rows, cols = x.shape
        out = _empty(rows, cols, device=x.device)
        clogit = _empty(rows, n, device=x.device)
        _check(lib.fx_process_feature_fwd(nx.ptr(x), nx.ld(x), rows, cols, n, nx.ptr(out), cols, nx.ptr(clogit), n,
                                          nx.stream()), "fx_process_feature_fwd")
        ctx.n = n
        ctx.save_for_backward(out)
        ctx.set_materialize_grads(False)   # an output without a gradient stays None (no zero fill)
        return out, clogit

    @staticmethod
    def backward(ctx, dout, dclogit):
        lib = nx.load()
        (out,) = ctx.saved_tensors
        rows, cols = out.shape
        if dout is None:
            dout = torch.zeros_like(out)
        dout = dout.contiguous()
        dclogit = None if dclogit is None else dclogit.contiguous()
        dx = _empty(rows, cols, device=out.device)
        _check(lib.fx_process_feature_bwd(nx.ptr(out), cols, nx.ptr(dout), cols, nx.ptr(dclogit), ctx.n, rows, cols,
                                          ctx.n, nx.ptr(dx), cols, nx.stream()), "fx_process_feature_bwd")
        return dx, None


def process_feature(x, n):
    """Returns (feature-with-probs, class logits) like the reference (its clogit is a view of the
    input; here it is a copy with the same values written by the same kernel)."""
    return ProcessFeatureFn.apply(_2d(x), n)


# ---------------------------------------------------------------------------
# L2 normalisation
# ---------------------------------------------------------------------------

class L2NormFn(torch.autograd.Function):
    """``F.normalize(dim=-1, eps=1e-12)`` (blocks.py:174)."""

    @staticmethod
    def forward(ctx, x):
        lib = nx.load()
        rows, cols = x.shape
        y = _empty(rows, cols, device=x.device)
        nrm = _empty(rows, device=x.device)
        _check(lib.fx_l2norm_fwd(nx.ptr(x), nx.ld(x), rows, cols, nx.ptr(y), cols, nx.ptr(nrm), nx.stream()),
               "fx_l2norm_fwd")
        ctx.save_for_backward(y, nrm)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = nx.load()
        y, nrm = ctx.saved_tensors
        dy = dy.contiguous()
        rows, cols = y.shape
        dx = _empty(rows, cols, device=y.device)
        _check(lib.fx_l2norm_bwd(nx.ptr(y), cols, nx.ptr(nrm), nx.ptr(dy), cols, rows, cols, nx.ptr(dx), cols,
                                 nx.stream()), "fx_l2norm_bwd")
        return dx


def l2_normalize(x):
    return L2NormFn.apply(_2d(x))


# ---------------------------------------------------------------------------
# Multi-head attention (nn.MultiheadAttention math)
# ---------------------------------------------------------------------------

class MHAFn(torch.autograd.Function):
    """``nn.MultiheadAttention`` forward/backward as used by SALayer/SCALayer
    (basic.py:442, 500, 513): in-projections, per-head softmax(QK^T/sqrt(hd))V, out_proj.
    ``w_packed`` (3E, E) is the packed in_proj_weight (kdim == E) or None with wq/wk/wv given."""

    @staticmethod
    def forward(ctx, q_in, k_in, v_in, w_packed, wq, wk, wv, b_in, wo, bo, nhead, drop_p=0.0, seed=0):
        lib = nx.load()
        dev = q_in.device
        Lq, Lk = q_in.shape[0], k_in.shape[0]
        E = wo.shape[0]
        if w_packed is not None:
            wq, wk, wv = w_packed[:E], w_packed[E:2 * E], w_packed[2 * E:]
        q = lin_fwd(q_in, wq, b_in[:E])
        k = lin_fwd(k_in, wk, b_in[E:2 * E])
        v = lin_fwd(v_in, wv, b_in[2 * E:])
        probs = _empty(nhead, Lq, Lk, device=dev)
        o = _empty(Lq, E, device=dev)
        ws = _ws(lib.fx_mha_core_workspace_floats(Lq, Lk, E, nhead), dev)
        _check(lib.fx_mha_core_fwd(nx.ptr(q), E, nx.ptr(k), E, nx.ptr(v), E, Lq, Lk, E, nhead, float(drop_p),
                                   int(seed), nx.ptr(probs), nx.ptr(o), E, nx.ptr(ws), nx.stream()), "fx_mha_core_fwd")
        out = lin_fwd(o, wo, bo)
        ctx.nhead = nhead
        ctx.drop = (float(drop_p), int(seed))
        ctx.packed = w_packed is not None
        ctx.save_for_backward(q_in, k_in, v_in, w_packed, wq, wk, wv, b_in, wo, bo, q, k, v, probs, o)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = nx.load()
        q_in, k_in, v_in, w_packed, wq, wk, wv, b_in, wo, bo, q, k, v, probs, o = ctx.saved_tensors
        nd = ctx.needs_input_grad
        dout = dout.contiguous()
        dev = dout.device
        Lq, Lk = q_in.shape[0], k_in.shape[0]
        E = wo.shape[0]
        nh = ctx.nhead
        dwo, dwo_ret = grad_target(wo, nd[8])
        dbo, dbo_ret = grad_target(bo, nd[9])
        d_o = lin_bwd(dout, o, wo, True, dwo, dbo)
        dq = _empty(Lq, E, device=dev)
        dk = _empty(Lk, E, device=dev)
        dv = _empty(Lk, E, device=dev)
        ws = _ws(lib.fx_mha_core_workspace_floats(Lq, Lk, E, nh), dev)
        _check(lib.fx_mha_core_bwd(nx.ptr(q), E, nx.ptr(k), E, nx.ptr(v), E, nx.ptr(probs), nx.ptr(d_o), E, Lq, Lk,
                                   E, nh, ctx.drop[0], ctx.drop[1], nx.ptr(dq), E, nx.ptr(dk), E, nx.ptr(dv), E,
                                   nx.ptr(ws), nx.stream()), "fx_mha_core_bwd")
        dbin, dbin_ret = grad_target(b_in, nd[7])
        rets = [None, None, None, None]
        if ctx.packed:
            dwp, rets[0] = grad_target(w_packed, nd[3])
            tq, tk, tv = (None, None, None) if dwp is None else (dwp[:E], dwp[E:2 * E], dwp[2 * E:])
        else:
            tq, rets[1] = grad_target(wq, nd[4])
            tk, rets[2] = grad_target(wk, nd[5])
            tv, rets[3] = grad_target(wv, nd[6])
        bq, bk, bv = (None, None, None) if dbin is None else (dbin[:E], dbin[E:2 * E], dbin[2 * E:])
        dq_in = lin_bwd(dq, q_in, wq, nd[0], tq, bq)
        dk_in = lin_bwd(dk, k_in, wk, nd[1], tk, bk)
        dv_in = lin_bwd(dv, v_in, wv, nd[2], tv, bv)
        return (dq_in, dk_in, dv_in, rets[0], rets[1], rets[2], rets[3], dbin_ret, dwo_ret, dbo_ret, None, None,
                None)


def mha(mod, query, key, value):
    """Run an nn.MultiheadAttention module's parameters through MHAFn; in training its dropout
    (on the attention probabilities) uses the kernels' counter-based mask."""
    if mod._qkv_same_embed_dim:
        args = (mod.in_proj_weight, None, None, None)
    else:
        args = (None, mod.q_proj_weight, mod.k_proj_weight, mod.v_proj_weight)
    p = float(mod.dropout) if mod.training else 0.0
    return MHAFn.apply(_2d(query), _2d(key), _2d(value), *args, mod.in_proj_bias, mod.out_proj.weight,
                       mod.out_proj.bias, mod.num_heads, p, dropout_seed() if p > 0 else 0)


# ---------------------------------------------------------------------------
# X2Y_map
# ---------------------------------------------------------------------------

class X2YFn(torch.autograd.Function):
    """``X2Y_map.forward`` (basic.py:349-389): returns (Y_out, attn_logit, attn).  ``rows`` = None
    (one video) or (x_off, y_off) host prefix lists of nvid stacked videos; logit / attn then pack
    each video's (ny_v, nx_v) block in video order."""

    @staticmethod
    def forward(ctx, X, Y, Xpos, Ypos, rows, wk, bk, wv, bv, wq, bq, wy, by, drop_p=0.0, seed=0, sinks=(None, None)):
        lib = nx.load()
        dev = X.device
        Nx, xdim = X.shape
        Ny, ydim = Y.shape
        Hd, outdim = wk.shape[0], wy.shape[0]
        if rows is None:
            nvid, xo, yo, na = 1, None, None, Ny * Nx
        else:
            xl, yl = rows
            nvid = len(xl) - 1
            xo, yo = nx.int_array(xl), nx.int_array(yl)
            na = sum((yl[v + 1] - yl[v]) * (xl[v + 1] - xl[v]) for v in range(nvid))
        out = _empty(Ny, outdim, device=dev)
        logit = _empty(na, device=dev)
        attn = _empty(na, device=dev)
        saved = _ws(lib.fx_x2y_saved_floats(Nx, xdim, Ny, ydim, Hd), dev)
        ws = _ws(lib.fx_x2y_workspace_floats(Nx, xdim, Ny, ydim, Hd, outdim, nvid, xo, yo), dev)
        xpc = 0 if Xpos is None else Xpos.shape[1]
        ypc = 0 if Ypos is None else Ypos.shape[1]
        _check(lib.fx_x2y_fwd(nx.ptr(X), nx.ld(X), Nx, xdim, nx.ptr(Xpos), nx.ld(Xpos), xpc,
                              nx.ptr(Y), nx.ld(Y), Ny, ydim, nx.ptr(Ypos), nx.ld(Ypos), ypc,
                              nx.ptr(wk), nx.ptr(bk), nx.ptr(wv), nx.ptr(bv), nx.ptr(wq), nx.ptr(bq),
                              nx.ptr(wy), nx.ptr(by), Hd, outdim, nvid, xo, yo, float(drop_p), int(seed),
                              nx.ptr(out), outdim, nx.ptr(logit), nx.ptr(attn), nx.ptr(saved), nx.ptr(ws),
                              nx.stream()), "fx_x2y_fwd")
        ctx.dims = (Nx, xdim, Ny, ydim, Hd, outdim, xpc, ypc)
        ctx.drop = (float(drop_p), int(seed))
        ctx.rows = rows
        ctx.has_pos = (Xpos is not None, Ypos is not None)
        ctx.sinks = sinks
        ctx.save_for_backward(X, Y, wk, bk, wv, bv, wq, bq, wy, by, attn, saved)
        ctx.set_materialize_grads(False)   # unused logit / attn gradients arrive as None (no zero fill)
        if rows is None:
            logit, attn = logit.view(Ny, Nx), attn.view(Ny, Nx)
        # the reference differentiates attn_logit only (its losses, blocks.py:372-377); attn feeds the
        # matching and eval (blocks.py:96, 243-281)
        ctx.mark_non_differentiable(attn)
        return out, logit, attn

    @staticmethod
    def backward(ctx, dout, dlogit, dattn):
        lib = nx.load()
        X, Y, wk, bk, wv, bv, wq, bq, wy, by, attn, saved = ctx.saved_tensors
        Nx, xdim, Ny, ydim, Hd, outdim, xpc, ypc = ctx.dims
        hx, hy = ctx.has_pos
        nd = ctx.needs_input_grad
        dev = X.device
        rows = ctx.rows
        if rows is None:
            nvid, xo, yo = 1, None, None
        else:
            nvid = len(rows[0]) - 1
            xo, yo = nx.int_array(rows[0]), nx.int_array(rows[1])
        dout = torch.zeros(Ny, outdim, device=dev) if dout is None else dout.contiguous()
        dlogit = None if dlogit is None else dlogit.contiguous()
        dattn = None if dattn is None else dattn.contiguous()
        dX = _empty(Nx, xdim, device=dev) if nd[0] else None
        dY = _empty(Ny, ydim, device=dev) if nd[1] else None
        # position gradients: fresh buffers, or accumulated into a shared PosGradSink (returned as None)
        dXp = dYp = None
        fx, fy = int(hx), int(hy)
        sx, sy = ctx.sinks
        if hx and nd[2]:
            if sx is not None:
                dXp, acc = sx.target((Nx, xpc), dev)
                fx |= 2 * acc
            else:
                dXp = _empty(Nx, xpc, device=dev)
        if hy and nd[3]:
            if sy is not None:
                dYp, acc = sy.target((Ny, ypc), dev)
                fy |= 2 * acc
            else:
                dYp = _empty(Ny, ypc, device=dev)
        tg = [grad_target(p, nd[5 + i]) for i, p in enumerate((wk, bk, wv, bv, wq, bq, wy, by))]
        bufs = [t[0] for t in tg]
        # the kernel needs every weight-gradient target; absent ones go to scratch
        bufs = [b if b is not None else torch.zeros_like(p) for b, p in zip(bufs, (wk, bk, wv, bv, wq, bq, wy, by))]
        ws = _ws(lib.fx_x2y_workspace_floats(Nx, xdim, Ny, ydim, Hd, outdim, nvid, xo, yo), dev)
        defer = _may_defer(tg)
        _check(lib.fx_x2y_bwd(nx.ptr(X), nx.ld(X), Nx, xdim, xpc, nx.ptr(Y), nx.ld(Y), Ny, ydim, ypc,
                              nx.ptr(wk), nx.ptr(wv), nx.ptr(wq), nx.ptr(wy), Hd, outdim, nvid, xo, yo,
                              ctx.drop[0], ctx.drop[1], nx.ptr(attn),
                              nx.ptr(saved), nx.ptr(dout), outdim, nx.ptr(dlogit), nx.ptr(dattn), nx.ptr(dX),
                              nx.ptr(dXp), nx.ptr(dY), nx.ptr(dYp), *[nx.ptr(t) for t in bufs], fx, fy,
                              nx.ptr(ws), int(defer), nx.ptr(device_status(dev)), nx.stream()), "fx_x2y_bwd")
        _queue_backward_status(dev)    # (the f2a core's grid-barrier timeout, FX_STATUS_X2Y_TIMEOUT)
        if defer:
            _defer_to_side(X, Y, saved, dout, ws, *bufs)
        if sx is not None:
            dXp = None
        if sy is not None:
            dYp = None
        return (dX, dY, dXp, dYp, None) + tuple(t[1] for t in tg) + (None, None, None)


def x2y(mod, X, Y, Xpos, Ypos, rows=None):
    p = float(mod.dropout.p) if mod.training else 0.0
    xp = None if Xpos is None else _2d(Xpos)
    yp = None if Ypos is None else _2d(Ypos)
    # a shared position-gradient buffer only when the op reads the sink's own output (not a view of it)
    sinks = (_sink_of(Xpos) if xp is Xpos else None, _sink_of(Ypos) if yp is Ypos else None)
    return X2YFn.apply(_2d(X), _2d(Y), xp, yp, rows, mod.X_K.weight, mod.X_K.bias, mod.X_V.weight, mod.X_V.bias,
                       mod.Y_Q.weight, mod.Y_Q.bias, mod.Y_W.weight, mod.Y_W.bias, p,
                       dropout_seed() if p > 0 else 0, sinks)


# ---------------------------------------------------------------------------
# MS-TCN stack
# ---------------------------------------------------------------------------

# fx_mstcn_params.fused_layers: the one-kernel MS-TCN layer (mstcn_fused.hip, weights in MFMA fragment
# order): on by default since round 4 (whole step 14.9 -> 14.5 ms);
# FX_MSTCN_FUSED_LAYERS=0 selects the two-GEMM layers (A/B knob)
# (2: also below one 32-row tile per CU, where the library would pick the two GEMMs -- tests)
MSTCN_FUSED_LAYERS = int(os.environ.get("FX_MSTCN_FUSED_LAYERS", "1"))


def _ptr_array(ts):
    return nx.array_type(ctypes.c_void_p, max(len(ts), 1))(*[nx.ptr(t) for t in ts])


class MSTCNFn(torch.autograd.Function):
    """Whole ``MSTCN.forward`` (basic.py:200-220) in one C call; training dropout on every layer's
    1x1 branch (basic.py:160) with the kernels' counter-based mask (seed in meta)."""

    @staticmethod
    def _unpack(meta, params):
        T, nvid, cin, F, cout, nl, ln, in_map, d0, dfac = meta[:10]
        it = iter(params)
        w_in = b_in = None
        if in_map:
            w_in, b_in = next(it), next(it)
        layers = []
        for _ in range(nl):
            lw = [next(it), next(it), next(it), next(it)]
            lw += [next(it), next(it)] if ln else [None, None]
            layers.append(lw)
        w_out, b_out = next(it), next(it)
        return w_in, b_in, layers, w_out, b_out

    @staticmethod
    def forward(ctx, x, meta, *params):
        lib = nx.load()
        T, nvid, cin, F, cout, nl, ln, in_map, d0, dfac, drop_p, seed, seq_off = meta
        w_in, b_in, layers, w_out, b_out = MSTCNFn._unpack(meta, params)
        keep = []
        prm = nx.MstcnParams()
        if seq_off is not None:     # ragged videos: host row offsets
            so = nx.int_array(seq_off)
            keep.append(so)
            prm.seq_off = ctypes.addressof(so)
        prm.cin, prm.F, prm.cout, prm.num_layers, prm.layernorm, prm.in_map = cin, F, cout, nl, int(ln), int(in_map)
        prm.dil0, prm.dil_factor = d0, dfac
        prm.w_in, prm.b_in = nx.ptr(w_in), nx.ptr(b_in)
        for field, k in (("w_dil", 0), ("b_dil", 1), ("w_pw", 2), ("b_pw", 3), ("ln_w", 4), ("ln_b", 5)):
            arr = _ptr_array([lw[k] for lw in layers])
            keep.append(arr)
            setattr(prm, field, ctypes.addressof(arr))
        prm.w_out, prm.b_out = nx.ptr(w_out), nx.ptr(b_out)
        prm.dropout, prm.seed = float(drop_p), int(seed)
        prm.fused_layers = int(MSTCN_FUSED_LAYERS)
        rows = x.shape[0]
        dev = x.device
        y = _empty(rows, cout, device=dev)
        saved = _ws(lib.fx_mstcn_saved_floats(ctypes.byref(prm), rows), dev)
        ws = _ws(lib.fx_mstcn_workspace_floats(ctypes.byref(prm), rows), dev)
        _check(lib.fx_mstcn_fwd(ctypes.byref(prm), nx.ptr(x), nx.ld(x), T, nvid, nx.ptr(y), cout, nx.ptr(saved),
                                nx.ptr(ws), nx.stream()), "fx_mstcn_fwd")
        ctx.meta = meta
        ctx.prm = prm
        ctx.keep = keep
        ctx.save_for_backward(x, saved, *params)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = nx.load()
        x, saved, *params = ctx.saved_tensors
        T, nvid, cin, F, cout, nl, ln, in_map, d0, dfac = ctx.meta[:10]
        dev = x.device
        dy = dy.contiguous()
        tg = [grad_target(p) for p in params]
        bufs = [t[0] for t in tg]
        w_in, b_in, layers, w_out, b_out = MSTCNFn._unpack(ctx.meta, bufs)
        g = nx.MstcnGrads()
        g.w_in, g.b_in = nx.ptr(w_in), nx.ptr(b_in)
        keep = []
        for field, k in (("w_dil", 0), ("b_dil", 1), ("w_pw", 2), ("b_pw", 3), ("ln_w", 4), ("ln_b", 5)):
            arr = _ptr_array([lw[k] for lw in layers])
            keep.append(arr)
            setattr(g, field, ctypes.addressof(arr))
        g.w_out, g.b_out = nx.ptr(w_out), nx.ptr(b_out)
        dx = _empty(*x.shape, device=dev) if ctx.needs_input_grad[0] else None
        ws = _ws(lib.fx_mstcn_workspace_floats(ctypes.byref(ctx.prm), x.shape[0]), dev)
        defer = _may_defer(tg)
        ctx.prm.side_defer = int(defer)
        _check(lib.fx_mstcn_bwd(ctypes.byref(ctx.prm), ctypes.byref(g), nx.ptr(x), nx.ld(x), T, nvid, nx.ptr(dy),
                                cout, nx.ptr(dx), nx.ld(dx), nx.ptr(saved), nx.ptr(ws), nx.stream()), "fx_mstcn_bwd")
        if defer:
            _defer_to_side(x, dy, saved, ws)
        return (dx, None) + tuple(t[1] for t in tg)


def mstcn(mod, x, T, nvid=1, seq_off=None):
    """Run a factmx.models.basic.MSTCN through MSTCNFn: nvid videos of T rows stacked in x, or the
    ragged videos of the host row-offset list seq_off (zero padding at every video's own ends)."""
    x2 = _2d(x)
    params = []
    if mod.in_map:
        params += [mod.conv_1x1.weight, mod.conv_1x1.bias]
    for lyr in mod.layers:
        params += [lyr.conv_dilated.weight, lyr.conv_dilated.bias, lyr.conv_1x1.weight, lyr.conv_1x1.bias]
        if lyr.norm is not None:
            params += [lyr.norm.weight, lyr.norm.bias]
    params += [mod.conv_out.weight, mod.conv_out.bias]
    ln = mod.layers[0].norm is not None if len(mod.layers) else False
    p = float(mod.dropout_rate) if (mod.training and mod.dropout_rate) else 0.0
    meta = (T, nvid, x2.shape[1], mod.hid_dim, mod.out_dim, mod.num_layers, bool(ln), bool(mod.in_map),
            mod.dilation0, mod.dilation_factor, p, dropout_seed() if p > 0 else 0,
            None if seq_off is None else tuple(int(v) for v in seq_off))
    return MSTCNFn.apply(x2, meta, *params)


class MSTCN2Fn(torch.autograd.Function):
    """Whole ``MSTCN2.forward`` (basic.py:263-281, MS-TCN++) in one C call: per layer the two dilated
    convs store into the halves of one concat buffer, the 1x1 fusion GEMM applies bias + ReLU (+ the
    training dropout of every layer but the last, counter-based mask from the seed in meta), one add
    forms the residual.  Backward: the input-gradient chain, then the weight gradients of all layers
    as batched GEMMs on the side stream.
    params: [w_in, b_in] (in_map) + w_d1 x L, b_d1 x L, w_d2 x L, b_d2 x L, w_fu x L, b_fu x L + w_out, b_out."""

    @staticmethod
    def _unpack(meta, params):
        nl, in_map = meta[5], meta[6]
        it = list(params)
        w_in = b_in = None
        if in_map:
            w_in, b_in, it = it[0], it[1], it[2:]
        groups = [it[k * nl:(k + 1) * nl] for k in range(6)]
        return w_in, b_in, groups, it[6 * nl], it[6 * nl + 1]

    @staticmethod
    def _prm(meta, params, keep, cls, grads=False):
        T, nvid, cin, F, cout, nl, in_map, dfac, drop_p, seed, seq_off = meta
        w_in, b_in, groups, w_out, b_out = MSTCN2Fn._unpack(meta, params)
        prm = cls()
        if not grads:
            prm.cin, prm.F, prm.cout, prm.num_layers, prm.in_map, prm.dil_factor = cin, F, cout, nl, int(in_map), dfac
            prm.dropout, prm.seed = float(drop_p), int(seed)
            if seq_off is not None:
                so = nx.int_array(seq_off)
                keep.append(so)
                prm.seq_off = ctypes.addressof(so)
        prm.w_in, prm.b_in = nx.ptr(w_in), nx.ptr(b_in)
        for field, grp in zip(("w_d1", "b_d1", "w_d2", "b_d2", "w_fu", "b_fu"), groups):
            arr = _ptr_array(grp)
            keep.append(arr)
            setattr(prm, field, ctypes.addressof(arr))
        prm.w_out, prm.b_out = nx.ptr(w_out), nx.ptr(b_out)
        return prm

    @staticmethod
    def forward(ctx, x, meta, *params):
        lib = nx.load()
        T, nvid, cout = meta[0], meta[1], meta[4]
        keep = []
        prm = MSTCN2Fn._prm(meta, params, keep, nx.Mstcn2Params)
        rows = x.shape[0]
        dev = x.device
        y = _empty(rows, cout, device=dev)
        saved = _ws(lib.fx_mstcn2_saved_floats(ctypes.byref(prm), rows), dev)
        ws = _ws(lib.fx_mstcn2_workspace_floats(ctypes.byref(prm), rows), dev)
        _check(lib.fx_mstcn2_fwd(ctypes.byref(prm), nx.ptr(x), nx.ld(x), T, nvid, nx.ptr(y), cout, nx.ptr(saved),
                                 nx.ptr(ws), nx.stream()), "fx_mstcn2_fwd")
        ctx.meta, ctx.prm, ctx.keep = meta, prm, keep
        ctx.save_for_backward(x, saved, *params)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = nx.load()
        x, saved, *params = ctx.saved_tensors
        T, nvid, cout = ctx.meta[0], ctx.meta[1], ctx.meta[4]
        dev = x.device
        dy = dy.contiguous()
        tg = [grad_target(p) for p in params]
        keep = []
        g = MSTCN2Fn._prm(ctx.meta, [t[0] for t in tg], keep, nx.Mstcn2Grads, grads=True)
        dx = _empty(*x.shape, device=dev) if ctx.needs_input_grad[0] else None
        ws = _ws(lib.fx_mstcn2_workspace_floats(ctypes.byref(ctx.prm), x.shape[0]), dev)
        defer = _may_defer(tg)
        ctx.prm.side_defer = int(defer)
        _check(lib.fx_mstcn2_bwd(ctypes.byref(ctx.prm), ctypes.byref(g), nx.ptr(x), nx.ld(x), T, nvid, nx.ptr(dy),
                                 cout, nx.ptr(dx), nx.ld(dx), nx.ptr(saved), nx.ptr(ws), nx.stream()), "fx_mstcn2_bwd")
        if defer:
            _defer_to_side(x, dy, saved, ws)
        return (dx, None) + tuple(t[1] for t in tg)


def mstcn2(mod, x, T, nvid=1, drop_p=0.0, seq_off=None):
    """Run a factmx.models.basic.MSTCN2 through MSTCN2Fn (x: (nvid*T, dim) rows, or the ragged videos of
    the host row-offset list seq_off)."""
    x2 = _2d(x)
    L = mod.num_layers
    params = [mod.conv_1x1_in.weight, mod.conv_1x1_in.bias] if mod.in_map else []
    params += [c.weight for c in mod.conv_dilated_1] + [c.bias for c in mod.conv_dilated_1]
    params += [c.weight for c in mod.conv_dilated_2] + [c.bias for c in mod.conv_dilated_2]
    params += [c.weight for c in mod.conv_fusion] + [c.bias for c in mod.conv_fusion]
    params += [mod.conv_out.weight, mod.conv_out.bias]
    meta = (T, nvid, x2.shape[1], mod.conv_out.weight.shape[1], mod.conv_out.weight.shape[0], L, bool(mod.in_map),
            int(mod.dilation_factor), float(drop_p), dropout_seed() if drop_p > 0 else 0,
            None if seq_off is None else tuple(int(v) for v in seq_off))
    return MSTCN2Fn.apply(x2, meta, *params)


# ---------------------------------------------------------------------------
# generic dilated Conv1d(k=3) (MSTCN2 / standalone DilatedResidualLayer pieces)
# ---------------------------------------------------------------------------

def _conv_operand(t, cin, dil, direction, T, trans):
    o = nx.Operand()
    o.ptr, o.ld = nx.ptr(t), nx.ld(t)
    o.trans = int(trans)
    o.conv_taps, o.conv_cin, o.conv_dil, o.conv_dir, o.seq_len = 3, cin, dil, direction, T
    return o


def _rows_operand(t, trans=False):
    o = nx.Operand()
    o.ptr, o.ld = nx.ptr(t), nx.ld(t)
    o.trans = int(trans)
    o.conv_dir = 1
    return o


def gemm(M, N, K, a, b, c, ldc, bias=None, relu=0, resid=None, alpha=1.0, beta=0.0, gate=None, c_tap_cin=0,
         split=1, c_last=None, batch=1, c_bs=0):
    lib = nx.load()
    d = nx.GemmDesc()
    d.M, d.N, d.K, d.batch = M, N, K, batch
    d.c_batch_stride = c_bs
    d.a, d.b = a, b
    d.c, d.ldc = nx.ptr(c), ldc
    d.alpha, d.beta = alpha, beta
    d.bias = nx.ptr(bias)
    d.resid, d.ld_resid = nx.ptr(resid), nx.ld(resid)
    d.gate, d.ld_gate = nx.ptr(gate), nx.ld(gate)
    d.relu, d.c_tap_cin = relu, c_tap_cin
    d.c_last_col = nx.ptr(c_last)
    d.split_k = split
    ws = None
    if split > 1:
        ws = _ws(lib.fx_gemm_workspace_floats(ctypes.byref(d)), c.device)
        d.workspace = nx.ptr(ws)
    _check(lib.fx_gemm(ctypes.byref(d), nx.stream()), "fx_gemm")
    return ws


def matmul_nt(x, w, alpha=1.0):
    """alpha * x . w^T for row-major x (M, K), w (N, K) without autograd (eval / matching paths):
    one fx_gemm launch instead of a hipBLASLt call and its host-side setup."""
    x, w = x.contiguous(), w.contiguous()
    M, K = x.shape
    N = w.shape[0]
    y = _empty(M, N, device=x.device)
    gemm(M, N, K, _rows_operand(x), _rows_operand(w), y, N, alpha=alpha)
    return y


def matmul_tn(a, b):
    """a^T . b for row-major a (K, M), b (K, N), no autograd: (M, N) via column-major operands."""
    a, b = a.contiguous(), b.contiguous()
    K, M = a.shape
    N = b.shape[1]
    y = _empty(M, N, device=a.device)
    gemm(M, N, K, _rows_operand(a, trans=True), _rows_operand(b, trans=True), y, N)
    return y


class Conv3Fn(torch.autograd.Function):
    """Conv1d(k=3, dilation d, padding d) on (T*nvid, C) rows as an implicit GEMM (basic.py:138, 237-245)."""

    @staticmethod
    def forward(ctx, x, w, b, dil, T):
        rows, cin = x.shape
        cout = w.shape[0]
        wf = w.permute(0, 2, 1).reshape(cout, 3 * cin).contiguous()       # [n][tap][c]
        y = _empty(rows, cout, device=x.device)
        gemm(rows, cout, 3 * cin, _conv_operand(x, cin, dil, 1, T, False), _rows_operand(wf), y, cout, bias=b)
        ctx.dil, ctx.T = dil, T
        ctx.save_for_backward(x, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, b = ctx.saved_tensors
        nd = ctx.needs_input_grad
        dy = dy.contiguous()
        rows, cin = x.shape
        cout = w.shape[0]
        dev = x.device
        dx = None
        if nd[0]:
            wb = w.permute(1, 2, 0).reshape(cin, 3 * cout).contiguous()   # [c][tap][n]
            dx = _empty(rows, cin, device=dev)
            gemm(rows, cin, 3 * cout, _conv_operand(dy, cout, ctx.dil, -1, ctx.T, False), _rows_operand(wb), dx, cin)
        dwb, dw_ret = grad_target(w, nd[1])
        dbb, db_ret = grad_target(b, nd[2])
        if dwb is not None:
            bop = _conv_operand(x, cin, ctx.dil, 1, ctx.T, True)
            ncol = 3 * cin + (1 if dbb is not None else 0)
            if dbb is not None:
                bop.ones_col = ncol
            split = max(1, min(16, rows // 256))
            gemm(cout, ncol, rows, _rows_operand(dy, trans=True), bop, dwb, 3 * cin, c_tap_cin=cin, split=split,
                 beta=1.0, c_last=dbb)
        elif dbb is not None:
            dbb += dy.sum(0)
        return dx, dw_ret, db_ret, None, None


def conv3(x, w, b, dil, T):
    return Conv3Fn.apply(_2d(x), w, b, dil, T)


# ---------------------------------------------------------------------------
# bidirectional GRU over segments
# ---------------------------------------------------------------------------

# Polls a BiGRU workgroup makes for a peer's step before it gives up (0: the library default,
# ~1 s).  Tests lower it to force the timeout path.
GRU_SPIN_MAX = 0
_status = {}


def device_status(dev):
    """The per-device int32 status word the kernels set on a failure they cannot report through a
    return code (FX_STATUS_GRU_TIMEOUT: a BiGRU workgroup gave up waiting for a peer, so that
    launch's outputs are wrong).  Read at the step's host read-back (status_raise)."""
    dev = torch.device(dev)
    if dev.type == "cuda" and dev.index is None:     # one word per physical device ("cuda" == "cuda:<current>")
        dev = torch.device("cuda", torch.cuda.current_device())
    t = _status.get(dev)
    if t is None:
        t = torch.zeros(4, dtype=torch.int32, device=dev)
        _status[dev] = t
    return t


def status_raise(value, dev):
    """Raise FactmxNativeError for a non-zero status word read back from the device (and clear it)."""
    if value:
        device_status(dev).zero_()
        _bwd_status.clear()       # (the same failure, possibly also seen by a backward-pass copy)
        raise nx.FactmxNativeError(f"device status {value}: {_status_text(value)} -- the outputs of this step "
                                   "are invalid")


def _status_text(value):
    parts = []
    if value & nx.STATUS_GRU_TIMEOUT:
        parts.append("a BiGRU workgroup timed out waiting for its peers (FX_STATUS_GRU_TIMEOUT)")
    if value & nx.STATUS_TOK_TIMEOUT:
        parts.append("a persistent token-kernel workgroup timed out at a grid barrier (FX_STATUS_TOK_TIMEOUT)")
    if value & nx.STATUS_X2Y_TIMEOUT:
        parts.append("an X2Y f2a-backward workgroup timed out at its grid barrier (FX_STATUS_X2Y_TIMEOUT)")
    return "; ".join(parts) or "unknown failure"


# Backward-pass status read-backs: a BiGRU backward writes the same status word as the forward, but
# after the forward's read-back was taken.  GRUFn.backward queues (once per backward pass) an end-of-
# pass callback that copies the word to pinned host memory behind an event -- ordered after every
# kernel of the backward, no host wait -- and the copy is checked at the next forward (or by
# check_device_status).  FusedAdam's update is guarded by the same word on the device, so the invalid
# gradients of such a step are never applied.
_bwd_status = []
_bwd_status_queued = False


def _queue_backward_status(dev):
    global _bwd_status_queued
    if _bwd_status_queued:
        return
    _bwd_status_queued = True
    stream = torch.cuda.current_stream(dev)

    def copy_status():
        global _bwd_status_queued
        _bwd_status_queued = False
        with torch.cuda.stream(stream):
            h = torch.empty(1, dtype=torch.int32, pin_memory=True)
            h.copy_(device_status(dev)[:1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        _bwd_status.append((h, ev, dev))
    torch.autograd.Variable._execution_engine.queue_callback(copy_status)


def resolve_backward_status(wait=False):
    """Raise FactmxNativeError if a kernel of an earlier BACKWARD pass set the status word.  Called
    between passes (a copy callback an aborted backward never ran must not block later ones).  At the
    start of a forward (wait=False) only copies that have already landed are checked -- waiting for the
    previous backward here would drain the device queue every step; FusedAdam's device-side guard
    covers the step in between.  check_device_status() waits (wait=True)."""
    global _bwd_status_queued
    _bwd_status_queued = False
    while _bwd_status:
        h, ev, dev = _bwd_status[0]
        if not wait and not ev.query():
            return
        _bwd_status.pop(0)
        ev.synchronize()
        if int(h[0]):
            _bwd_status.clear()
            device_status(dev).zero_()
            raise nx.FactmxNativeError(
                f"device status {int(h[0])}: {_status_text(int(h[0]))} in the BACKWARD pass of the previous step "
                "-- its gradients are invalid (a factmx FusedAdam step on them was skipped on the device)")


def check_device_status(dev=None):
    """Synchronous check of the status word (e.g. after the last backward of a run)."""
    from .models import vloss
    vloss.resolve_pending()
    resolve_backward_status(wait=True)
    dev = torch.device("cuda", torch.cuda.current_device()) if dev is None else torch.device(dev)
    status_raise(int(device_status(dev)[0].item()), dev)


class GRUFn(torch.autograd.Function):
    """One bidirectional ``nn.GRU`` layer (blocks.py:401,432) on (S, In) rows -> (S, 2Hh).
    ``seq_off`` = None (one sequence) or the host prefix list of several sequences stacked by
    rows (one per video), run concurrently by the kernel.  ``relu``: the output is relu(GRU(x)) (the
    UpdateBlockTDU's torch.relu, blocks.py:432, written by the recurrence kernel, its backward gate applied
    to dout by the backward kernel: no separate launch or autograd node either way)."""

    @staticmethod
    def forward(ctx, x, seq_off, relu, w_ih, w_hh, b_ih, b_hh, w_ih_r, w_hh_r, b_ih_r, b_hh_r):
        lib = nx.load()
        S, In = x.shape
        Hh = w_hh.shape[1]
        dev = x.device
        nq = 1 if seq_off is None else len(seq_off) - 1
        so = None if seq_off is None else nx.int_array(seq_off)
        out = _empty(S, 2 * Hh, device=dev)
        saved = _ws(lib.fx_gru_saved_floats(S, Hh), dev)
        ws = _ws(lib.fx_gru_workspace_floats(S, nq, In, Hh), dev)
        _check(lib.fx_gru_bidir_fwd(nx.ptr(x), nx.ld(x), S, nq, so, In, Hh, nx.ptr(w_ih), nx.ptr(w_hh), nx.ptr(b_ih),
                                    nx.ptr(b_hh), nx.ptr(w_ih_r), nx.ptr(w_hh_r), nx.ptr(b_ih_r), nx.ptr(b_hh_r),
                                    nx.ptr(out), 2 * Hh, int(bool(relu)), nx.ptr(saved), nx.ptr(ws),
                                    nx.ptr(device_status(dev)), GRU_SPIN_MAX, nx.stream()), "fx_gru_bidir_fwd")
        ctx.seq_off = seq_off
        ctx.relu = bool(relu)
        ctx.save_for_backward(x, w_ih, w_hh, b_ih, b_hh, w_ih_r, w_hh_r, b_ih_r, b_hh_r, saved,
                              out if relu else None)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = nx.load()
        x, *w, saved, y = ctx.saved_tensors
        w_ih, w_hh, _, _, w_ih_r, w_hh_r, _, _ = w
        dout = dout.contiguous()
        S, In = x.shape
        Hh = w_hh.shape[1]
        dev = x.device
        nd = ctx.needs_input_grad
        seq_off = ctx.seq_off
        nq = 1 if seq_off is None else len(seq_off) - 1
        so = None if seq_off is None else nx.int_array(seq_off)
        dx = _empty(S, In, device=dev) if nd[0] else None
        tg = [grad_target(p, nd[3 + i]) for i, p in enumerate(w)]
        bufs = [t[0] for t in tg]
        ws = _ws(lib.fx_gru_workspace_floats(S, nq, In, Hh), dev)
        _check(lib.fx_gru_bidir_bwd(nx.ptr(x), nx.ld(x), S, nq, so, In, Hh, nx.ptr(w_ih), nx.ptr(w_hh), nx.ptr(w_ih_r),
                                    nx.ptr(w_hh_r), nx.ptr(saved), nx.ptr(dout), 2 * Hh, nx.ptr(y), 2 * Hh,
                                    nx.ptr(dx), nx.ld(dx),
                                    *[nx.ptr(t) for t in bufs], nx.ptr(ws), nx.ptr(device_status(dev)), GRU_SPIN_MAX,
                                    nx.stream()), "fx_gru_bidir_bwd")
        _queue_backward_status(dev)
        return (dx, None, None) + tuple(t[1] for t in tg)


def gru(mod, x, seq_off=None, relu=False):
    """Run an ``nn.GRU(bidirectional=True)`` module's parameters layer by layer through GRUFn; in
    training, ``mod.dropout`` on every layer's output but the last (nn.GRU's inter-layer dropout).
    ``relu``: relu of the last layer's output, in the kernel (see GRUFn)."""
    assert mod.bidirectional and not mod.batch_first
    h = _2d(x)
    p_drop = float(mod.dropout) if (mod.training and mod.num_layers > 1) else 0.0
    for layer in range(mod.num_layers):
        if layer and p_drop:
            h = torch.nn.functional.dropout(h, p_drop, True)
        p = [getattr(mod, f"{n}_l{layer}{s}") for s in ("", "_reverse")
             for n in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")]
        h = GRUFn.apply(h, seq_off, relu and layer == mod.num_layers - 1, *p)
    return h


# ---------------------------------------------------------------------------
# Temporal down/up-sampling
# ---------------------------------------------------------------------------

def segments_from_probs(x2d, col0, ncls):
    """Device argmax + run-length boundaries; returns (S, seg_id, start, end) with one host read of S."""
    lib = nx.load()
    T = x2d.shape[0]
    dev = x2d.device
    buf = torch.empty(4 * T + 1, device=dev, dtype=torch.int32)
    pred, seg_id, st, en = buf[:T], buf[T:2 * T], buf[2 * T:3 * T], buf[3 * T:4 * T]
    ns = buf[4 * T:]
    _check(lib.fx_segments_from_probs(nx.ptr(x2d), nx.ld(x2d), col0, ncls, T, 1, None, nx.ptr(pred), nx.ptr(seg_id),
                                      nx.ptr(st), nx.ptr(en), nx.ptr(ns), nx.stream()), "fx_segments_from_probs")
    S = int(ns.item())
    return S, seg_id, st[:S], en[:S]


_NS_HOST = {}


def segments_from_probs_batched(x2d, col0, ncls, f_off, while_waiting=None):
    """``segments_from_probs`` for the videos stacked in x2d (host frame-row prefix list f_off, ragged
    lengths allowed), with ONE host read of all segment counts.  Returns (S list, per-video local
    (seg_id, start, end) views, global (seg_id, start, end) over the stacked frame rows /
    concatenated segments).  ``while_waiting``: host work that does not need S, run after the counts'
    copy is enqueued and before the host waits for it (the device is still working up to this block)."""
    lib = nx.load()
    dev = x2d.device
    nvid = len(f_off) - 1
    n = f_off[-1]
    ro = nx.int_array(f_off)
    buf = torch.empty(4 * n + nvid, device=dev, dtype=torch.int32)
    pred, seg_id, st, en = buf[:n], buf[n:2 * n], buf[2 * n:3 * n], buf[3 * n:4 * n]
    ns = buf[4 * n:]
    _check(lib.fx_segments_from_probs(nx.ptr(x2d), nx.ld(x2d), col0, ncls, 0, nvid, ro, nx.ptr(pred), nx.ptr(seg_id),
                                      nx.ptr(st), nx.ptr(en), nx.ptr(ns), nx.stream()), "fx_segments_from_probs")
    nh = _NS_HOST.get(nvid)
    if nh is None:
        nh = _NS_HOST[nvid] = torch.empty(nvid, dtype=torch.int32, pin_memory=True)
    nh.copy_(ns, non_blocking=True)
    ready = torch.cuda.Event()
    ready.record()
    if while_waiting is not None:
        while_waiting()
    ready.synchronize()
    S = nh.tolist()
    tot = sum(S)
    g = torch.empty(n + 2 * tot, device=dev, dtype=torch.int32)
    gid, gst, gen = g[:n], g[n:n + tot], g[n + tot:]
    _check(lib.fx_segments_globalize(nvid, 0, ro, nx.int_array(S), nx.ptr(seg_id), nx.ptr(st), nx.ptr(en), nx.ptr(gid),
                                     nx.ptr(gst), nx.ptr(gen), nx.stream()), "fx_segments_globalize")
    local = [(seg_id[f_off[v]:f_off[v + 1]], st[f_off[v]:f_off[v] + S[v]], en[f_off[v]:f_off[v] + S[v]])
             for v in range(nvid)]
    return S, local, (gid, gst, gen)


class SegMeanFn(torch.autograd.Function):
    """``feature_frame2seg`` (basic.py:615-625): index_add over frames / segment length."""

    @staticmethod
    def forward(ctx, x, seg_id, st, en):
        lib = nx.load()
        S = st.shape[0]
        T, C = x.shape
        y = _empty(S, C, device=x.device)
        _check(lib.fx_seg_mean_fwd(nx.ptr(x), nx.ld(x), nx.ptr(st), nx.ptr(en), S, C, nx.ptr(y), C, nx.stream()),
               "fx_seg_mean_fwd")
        ctx.save_for_backward(seg_id, st, en)
        ctx.T = T
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = nx.load()
        seg_id, st, en = ctx.saved_tensors
        dy = dy.contiguous()
        C = dy.shape[1]
        dx = _empty(ctx.T, C, device=dy.device)
        _check(lib.fx_seg_mean_bwd(nx.ptr(dy), C, nx.ptr(seg_id), nx.ptr(st), nx.ptr(en), ctx.T, C, nx.ptr(dx), C, 0,
                                   nx.stream()), "fx_seg_mean_bwd")
        return dx, None, None, None


def seg_sum_rows(x, st, en):
    lib = nx.load()
    S = st.shape[0]
    C = x.shape[1]
    y = _empty(S, C, device=x.device)
    _check(lib.fx_seg_sum_rows(nx.ptr(x), nx.ld(x), nx.ptr(st), nx.ptr(en), S, C, nx.ptr(y), C, 0, nx.stream()),
           "fx_seg_sum_rows")
    return y


class SegMergeFn(torch.autograd.Function):
    """``temporal_upsample`` (blocks.py:439-447): relu(sf_merge(cat[seg[seg_id], frame])).
    The segment->frame gather is the A-operand row gather of the GEMM."""

    @staticmethod
    def forward(ctx, seg, frame, seg_id, st, en, w, b):
        T = frame.shape[0]
        Fs, H = seg.shape[1], frame.shape[1]
        N = w.shape[0]
        y = _empty(T, N, device=frame.device)
        a = _rows_operand(seg)
        a.rows0 = nx.ptr(seg_id)
        a.ptr1, a.ld1, a.k_split = nx.ptr(frame), nx.ld(frame), Fs
        gemm(T, N, Fs + H, a, _rows_operand(w), y, N, bias=b, relu=1)
        ctx.save_for_backward(seg, frame, st, en, w, b, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = nx.load()
        seg, frame, st, en, w, b, y = ctx.saved_tensors
        nd = ctx.needs_input_grad
        dy = dy.contiguous()
        T, N = y.shape
        Fs = seg.shape[1]
        dz = _empty(T, N, device=dy.device)
        _check(lib.fx_relu_bwd(nx.ptr(dy), N, nx.ptr(y), N, T, N, nx.ptr(dz), N, nx.stream()), "fx_relu_bwd")
        dzs = seg_sum_rows(dz, st, en)                        # gather backward folded before the GEMM
        dwb, dw_ret = grad_target(w, nd[5])
        dbb, db_ret = grad_target(b, nd[6])
        dseg = lin_bwd(dzs, seg, w[:, :Fs], nd[0], None if dwb is None else dwb[:, :Fs])
        dframe = lin_bwd(dz, frame, w[:, Fs:], nd[1], None if dwb is None else dwb[:, Fs:], dbb)
        return dseg, dframe, None, None, None, dw_ret, db_ret


# ---------------------------------------------------------------------------
# elementwise
# ---------------------------------------------------------------------------

def add_(a, b):
    """a += b on device (same shape)."""
    lib = nx.load()
    rows, cols = a.shape
    _check(lib.fx_add(nx.ptr(b), nx.ld(b), None, 0, rows, cols, nx.ptr(a), nx.ld(a), 1, nx.stream()), "fx_add")
    return a


# ---------------------------------------------------------------------------
# Action-token decoders (SCADecoder / SADecoder), whole stack per call
# ---------------------------------------------------------------------------

def _decoder_slots(mod):
    """Map an SCADecoder / SADecoder onto fx_decoder_params: returns (meta, params, slots) where
    ``params`` are the unique parameter tensors (autograd inputs) and ``slots[field]`` lists, per
    layer (or once for the global fields), (param index, element offset)."""
    layers = list(mod.layers)
    cross = hasattr(layers[0], "self_attn")
    params, index = [], {}

    def slot(t, off=0):
        if t is None:
            return None
        k = id(t)
        if k not in index:
            index[k] = len(params)
            params.append(t)
        return (index[k], off)

    slots = {f: [] for f in nx.DECODER_LAYER_FIELDS}
    for lyr in layers:
        sa = lyr.self_attn if cross else lyr.multihead_attn
        if not sa._qkv_same_embed_dim:
            raise NotImplementedError("self-attention with kdim != embed_dim")
        A = sa.embed_dim
        slots["sa_in_w"].append(slot(sa.in_proj_weight))
        slots["sa_in_b"].append(slot(sa.in_proj_bias))
        slots["sa_out_w"].append(slot(sa.out_proj.weight))
        slots["sa_out_b"].append(slot(sa.out_proj.bias))
        if cross:
            ca = lyr.multihead_attn
            if ca._qkv_same_embed_dim:
                w = ca.in_proj_weight
                qw, kw, vw = slot(w, 0), slot(w, A * A), slot(w, 2 * A * A)
            else:
                qw, kw, vw = slot(ca.q_proj_weight), slot(ca.k_proj_weight), slot(ca.v_proj_weight)
            slots["ca_q_w"].append(qw)
            slots["ca_k_w"].append(kw)
            slots["ca_v_w"].append(vw)
            slots["ca_in_b"].append(slot(ca.in_proj_bias))
            slots["ca_out_w"].append(slot(ca.out_proj.weight))
            slots["ca_out_b"].append(slot(ca.out_proj.bias))
            slots["ln_ca_w"].append(slot(lyr.norm2.weight))
            slots["ln_ca_b"].append(slot(lyr.norm2.bias))
            ln_ff = lyr.norm3
        else:
            for f in ("ca_q_w", "ca_k_w", "ca_v_w", "ca_in_b", "ca_out_w", "ca_out_b", "ln_ca_w", "ln_ca_b"):
                slots[f].append(None)
            ln_ff = lyr.norm2
        slots["ff1_w"].append(slot(lyr.linear1.weight))
        slots["ff1_b"].append(slot(lyr.linear1.bias))
        slots["ff2_w"].append(slot(lyr.linear2.weight))
        slots["ff2_b"].append(slot(lyr.linear2.bias))
        slots["ln_sa_w"].append(slot(lyr.norm1.weight))
        slots["ln_sa_b"].append(slot(lyr.norm1.bias))
        slots["ln_ff_w"].append(slot(ln_ff.weight))
        slots["ln_ff_b"].append(slot(ln_ff.bias))
    norm = mod.norm
    gl = {"fn_w": slot(norm.weight) if norm is not None else None,
          "fn_b": slot(norm.bias) if norm is not None else None,
          "out_w": slot(mod.out_linear.weight), "out_b": slot(mod.out_linear.bias)}
    lyr0 = layers[0]
    sa0 = lyr0.self_attn if cross else lyr0.multihead_attn
    eps = lyr0.norm1.eps
    meta = dict(A=sa0.embed_dim, FF=lyr0.linear1.out_features, nhead=sa0.num_heads, num_layers=len(layers),
                cross=int(cross), Hm=(lyr0.multihead_attn.kdim if cross else 0), out_dim=mod.out_linear.out_features,
                final_norm=int(norm is not None), eps=float(eps))
    return meta, params, slots, gl


def _fill_decoder_struct(st, slots, gl, tensors, keep):
    """Point every field of a DecoderParams / DecoderGrads at ``tensors[idx] + off``."""
    def addr(s):
        if s is None or tensors[s[0]] is None:
            return None
        return tensors[s[0]].data_ptr() + 4 * s[1]
    for f, lst in slots.items():
        arr = nx.array_type(ctypes.c_void_p, max(len(lst), 1))(*[addr(s) for s in lst])
        keep.append(arr)
        setattr(st, f, ctypes.addressof(arr))
    for f, s in gl.items():
        setattr(st, f, addr(s))


class DecoderFn(torch.autograd.Function):
    """SCADecoder.forward (basic.py:542-557) / SADecoder.forward (basic.py:578-593) in one C call
    per direction (fx_decoder_fwd / fx_decoder_bwd)."""

    @staticmethod
    def _set_call(prm, call):
        """Per-call fields (dropout p's and seed, ragged memory offsets) of the cached param struct."""
        pd, pa, seed, mem_off = call[:4]
        prm.dropout, prm.attn_dropout, prm.seed = pd, pa, seed
        prm.mem_off = None if mem_off is None else ctypes.addressof(mem_off)

    @staticmethod
    def forward(ctx, tgt, qpos, mem, mpos, spec, nvid, call, *params):
        lib = nx.load()
        meta, slots, gl, cache = spec
        prm = cache.get("prm")
        key = tuple(p.data_ptr() for p in params)
        if prm is None or cache.get("key") != key:
            prm = nx.DecoderParams(**meta)
            keep = []
            _fill_decoder_struct(prm, slots, gl, params, keep)
            cache.update(prm=prm, key=key, keep=keep)
        DecoderFn._set_call(prm, call)
        prm.status = nx.ptr(device_status(tgt.device))
        ctx.call = call
        R = tgt.shape[0]
        T = mem.shape[0] if mem is not None else 0
        hq, hm = int(qpos is not None), int(mpos is not None)
        dev = tgt.device
        out = _empty(R, meta["out_dim"], device=dev)
        saved = _ws(lib.fx_decoder_saved_floats(ctypes.byref(prm), R, T, nvid, hq, hm), dev)
        ws = _ws(lib.fx_decoder_workspace_floats(ctypes.byref(prm), R, T, nvid, hq, hm), dev)
        _check(lib.fx_decoder_fwd(ctypes.byref(prm), nx.ptr(tgt), nx.ld(tgt), R, nx.ptr(qpos), nx.ld(qpos),
                                  nx.ptr(mem), nx.ld(mem), T, nvid, nx.ptr(mpos), nx.ld(mpos), nx.ptr(out),
                                  nx.ld(out), nx.ptr(saved), nx.ptr(ws), nx.stream()), "fx_decoder_fwd")
        ctx.spec = spec
        ctx.flags = (hq, hm, T, nvid)
        ctx.save_for_backward(tgt, qpos, mem, mpos, saved, *params)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = nx.load()
        tgt, qpos, mem, mpos, saved, *params = ctx.saved_tensors
        meta, slots, gl, cache = ctx.spec
        hq, hm, T, nvid = ctx.flags
        nd = ctx.needs_input_grad
        dev = dout.device
        dout = dout.contiguous()
        R = tgt.shape[0]
        tg = [grad_target(p, nd[7 + i]) for i, p in enumerate(params)]
        bufs = [t[0] for t in tg]
        gkey = tuple(0 if b is None else b.data_ptr() for b in bufs)
        g = cache.get("grads")
        if g is None or cache.get("gkey") != gkey:
            g = nx.DecoderGrads()
            keep = []
            _fill_decoder_struct(g, slots, gl, bufs, keep)
            cache.update(grads=g, gkey=gkey, gkeep=keep)
        prm = cache["prm"]
        DecoderFn._set_call(prm, ctx.call)        # the module may have run again since this forward
        prm.status = nx.ptr(device_status(dev))
        A = meta["A"]
        dtgt = _empty(R, A, device=dev) if nd[0] else None
        dqpos, sink = None, ctx.call[4]
        prm.dqpos_accumulate = 0
        if hq and nd[1]:
            if sink is not None:     # accumulated into the table's shared buffer (PosGradSink)
                dqpos, prm.dqpos_accumulate = sink.target((R, A), dev)
            else:
                dqpos = _empty(R, A, device=dev)
        dmem = _empty(*mem.shape, device=dev) if (mem is not None and nd[2]) else None
        dmpos = _empty(*mpos.shape, device=dev) if (hm and nd[3]) else None
        ws = _ws(lib.fx_decoder_workspace_floats(ctypes.byref(prm), R, T, nvid, hq, hm), dev)
        # the token linears' weight gradients (and, cross-attention decoders, the frame-memory K/V one)
        # stay on the side stream
        defer = _may_defer(tg)
        prm.side_defer = int(defer)
        _check(lib.fx_decoder_bwd(ctypes.byref(prm), ctypes.byref(g), nx.ptr(tgt), nx.ld(tgt), R, nx.ptr(qpos),
                                  nx.ptr(mem), nx.ld(mem), T, nvid, nx.ptr(mpos), nx.ld(mpos), nx.ptr(dout),
                                  nx.ld(dout),
                                  nx.ptr(dtgt), nx.ld(dtgt), nx.ptr(dqpos), nx.ptr(dmem), nx.ld(dmem), nx.ptr(dmpos),
                                  nx.ld(dmpos), nx.ptr(saved), nx.ptr(ws), nx.stream()), "fx_decoder_bwd")
        _queue_backward_status(dev)    # (a token-kernel barrier timeout in this backward, FX_STATUS_TOK_TIMEOUT)
        if defer:   # (dout too: the output linear's weight gradient reads it on the side stream)
            _defer_to_side(tgt, mem, mpos, saved, ws, dout)
        if sink is not None:
            dqpos = None
        return (dtgt, dqpos, dmem, dmpos, None, None, None) + tuple(t[1] for t in tg)


def decoder(mod, tgt, memory=None, pos=None, query_pos=None, nvid=1, mem_off=None):
    """Run an SCADecoder (memory given) or SADecoder through DecoderFn; returns (R, out_dim).
    ``nvid`` videos stacked by rows: tokens split evenly, memory frames evenly or by the host prefix
    list ``mem_off`` (ragged videos).  In training the layers' dropout runs inside the kernels
    (counter-based masks from one drawn seed)."""
    spec = getattr(mod, "_fx_spec", None)
    if spec is None:
        meta, params, slots, gl = _decoder_slots(mod)
        spec = (meta, slots, gl, {})
        mod._fx_spec = spec
        mod._fx_params = params
    params = mod._fx_params
    t2 = _2d(tgt)
    qp = None if query_pos is None else _2d(query_pos).contiguous()
    mem = None if memory is None else _2d(memory)
    mp = None if pos is None else _2d(pos)
    from .models.basic import decoder_dropout
    pd, pa = decoder_dropout(mod) if mod.training else (0.0, 0.0)
    seed = dropout_seed() if (pd > 0 or pa > 0) else 0
    off = None if (mem_off is None or memory is None) else nx.int_array(mem_off)
    sink = _sink_of(query_pos) if qp is query_pos else None
    return DecoderFn.apply(t2, qp, mem, mp, spec, int(nvid), (float(pd), float(pa), seed, off, sink), *params)


# ---------------------------------------------------------------------------
# Fused loss terms (fx_class_loss_*, fx_attn_loss_*)
# ---------------------------------------------------------------------------

_loss_ws_cache = {}


def _loss_ws(dev):
    t = _loss_ws_cache.get(dev)
    if t is None:
        t = torch.empty(nx.load().fx_loss_workspace_floats(), device=dev)
        _loss_ws_cache[dev] = t
    return t


class ClassLossFn(torch.autograd.Function):
    """c_ce * sum_r CE(x_r; target_r, w) + c_sm * sum smooth terms of x (loss.py:8-18, 246-277) as one
    scalar; hard int64 labels y or soft target rows z (R, C)."""

    @staticmethod
    def forward(ctx, x, y, z, w, c_ce, c_sm):
        lib = nx.load()
        R, C = x.shape
        dev = x.device
        lse = _empty(R, device=dev)
        out = _empty(1, device=dev)
        _check(lib.fx_class_loss_fwd(nx.ptr(x), x.stride(0), x.stride(1), R, C, nx.ptr(y), nx.ptr(z), nx.ptr(w),
                                     float(c_ce), float(c_sm), nx.ptr(lse), nx.ptr(out), nx.ptr(_loss_ws(dev)),
                                     nx.stream()), "fx_class_loss_fwd")
        ctx.c = (float(c_ce), float(c_sm))
        ctx.save_for_backward(x, y, z, w, lse)
        return out.reshape(())

    @staticmethod
    def backward(ctx, g):
        lib = nx.load()
        x, y, z, w, lse = ctx.saved_tensors
        R, C = x.shape
        g = g.reshape(1).contiguous()
        dx = _empty(R, C, device=x.device)
        _check(lib.fx_class_loss_bwd(nx.ptr(x), x.stride(0), x.stride(1), R, C, nx.ptr(y), nx.ptr(z), nx.ptr(w),
                                     nx.ptr(lse), ctx.c[0], ctx.c[1], nx.ptr(g), nx.ptr(dx), nx.stream()),
               "fx_class_loss_bwd")
        return dx, None, None, None, None, None


class AttnLossFn(torch.autograd.Function):
    """c_xe * cross-attention CE over the matched columns (loss.py:209-244) + c_sm * smooth terms of
    the attention logits, as one scalar.  ``L`` (R, Q) may be any strided view."""

    @staticmethod
    def forward(ctx, L, z, a_idx, s_idx, sweight, axis, c_xe, c_sm):
        lib = nx.load()
        R, Q = L.shape
        dev = L.device
        K, S = len(a_idx), z.shape[1]
        ai, si, sw = nx.int_array(a_idx), nx.int_array(s_idx), nx.float_array(sweight)
        lse_sel = _empty(max(R if axis == 1 else K, 1), device=dev)
        lse_full = _empty(R, device=dev) if c_sm else None
        colz = _empty(max(K, 1), device=dev) if axis == 0 else None
        out = _empty(1, device=dev)
        _check(lib.fx_attn_loss_fwd(nx.ptr(L), L.stride(0), L.stride(1), R, Q, K, ai, si, sw, nx.ptr(z), S, axis,
                                    float(c_xe), float(c_sm), nx.ptr(lse_sel), nx.ptr(lse_full), nx.ptr(colz),
                                    nx.ptr(out), nx.ptr(_loss_ws(dev)), nx.stream()), "fx_attn_loss_fwd")
        ctx.args = (list(a_idx), list(s_idx), list(sweight), axis, float(c_xe), float(c_sm))
        ctx.save_for_backward(L, z, lse_sel, lse_full, colz)
        return out.reshape(())

    @staticmethod
    def backward(ctx, g):
        lib = nx.load()
        L, z, lse_sel, lse_full, colz = ctx.saved_tensors
        a_idx, s_idx, sweight, axis, c_xe, c_sm = ctx.args
        R, Q = L.shape
        g = g.reshape(1).contiguous()
        # gradient in the input view's memory order (a transposed view gets a transposed buffer)
        dL = _empty(Q, R, device=L.device).t() if (L.stride(0) == 1 and Q > 1) else _empty(R, Q, device=L.device)
        _check(lib.fx_attn_loss_bwd(nx.ptr(L), L.stride(0), L.stride(1), R, Q, len(a_idx), nx.int_array(a_idx),
                                    nx.int_array(s_idx), nx.float_array(sweight), nx.ptr(z), z.shape[1], axis,
                                    nx.ptr(lse_sel), nx.ptr(lse_full), nx.ptr(colz), c_xe, c_sm, nx.ptr(g),
                                    nx.ptr(dL), dL.stride(0), dL.stride(1), nx.stream()), "fx_attn_loss_bwd")
        return dL, None, None, None, None, None, None, None
