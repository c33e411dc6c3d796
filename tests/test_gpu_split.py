"""FX_PREC_F32S: fp32 GEMM arithmetic on the bf16 matrix cores (3-piece bf16 split of every fp32
operand, 6 piece products summed in the fp32 accumulator; gemm_f32.hip gemm_split_wide8_kernel).

Checked against the float64 product of the SAME fp32 inputs, next to the native f32-MFMA kernel on
the same shapes: the split kernel's error must stay at fp32 level (within 2x the native kernel's
max error, plus a K-scaled fp32 floor), on every operand kind the mode takes (row-major A and B,
B stored transposed, the implicit dilated conv with per-video zero padding, a concatenated A,
split-K, the bias / ReLU / residual epilogue).  The 2-piece variant (FX_PREC_F32S2) is checked to
really be a different, coarser arithmetic (so the 3-piece result is not the native kernel by
accident).  At model level the north-star step (FACT_CLIP, T=4096, 2 videos, lockstep) in this mode
is held to the SAME parity bounds as the fp32 path against the fp64 oracle."""
import math

import pytest
import torch

from factmx import functional as fxf
from factmx import native as nx

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g, dtype=torch.float64) * scale).float().double()


def _rows(t, ld=None):
    o = nx.Operand()
    o.ptr = nx.ptr(t)
    o.ld = ld or t.shape[-1]
    o.conv_dir = 1
    return o


def _run(prec, M, N, K, a_fn, b_fn, split=1, **kw):
    c = torch.zeros(M, N, device=DEV)
    with fxf.gemm_precision(prec):
        fxf.gemm(M, N, K, a_fn(), b_fn(), c, N, split=split, **kw)
    torch.cuda.synchronize()
    return c.double().cpu()


def _check(ref, M, N, K, a_fn, b_fn, split=1, **kw):
    got32 = _run("fp32", M, N, K, a_fn, b_fn, split, **kw)
    got_s = _run("fp32s", M, N, K, a_fn, b_fn, split, **kw)
    got_s2 = _run("fp32s2", M, N, K, a_fn, b_fn, split, **kw)
    e32 = (got32 - ref).abs().max().item()
    es = (got_s - ref).abs().max().item()
    es2 = (got_s2 - ref).abs().max().item()
    scale = ref.abs().max().item()
    print(f"max |err|: native f32 {e32:.3e}  split-3 {es:.3e}  split-2 {es2:.3e}  (|ref| max {scale:.3e})")
    assert es <= 2.0 * e32 + 2 ** -24 * math.sqrt(K) * scale, (es, e32)
    assert es2 > 4 * es, (es2, es)          # the 3-piece split is not the 2-piece (or bf16) arithmetic
    assert nx.load().fx_get_stream_precision(nx.stream()) == nx.load().fx_get_default_precision()


@pytest.mark.parametrize("M,N,K,split,epi,bt", [(8192, 256, 256, 1, "plain", False),
                                                (8192, 256, 768, 1, "bias_relu_resid", False),
                                                (8000, 256, 512, 1, "plain", False),
                                                (4096, 512, 1024, 2, "plain", False),
                                                (8192, 512, 2048, 1, "bias_relu_resid", False),
                                                (8192, 256, 256, 1, "plain", True),
                                                (8000, 512, 3072, 1, "plain", True)])
def test_split_gemm_fp32_accuracy(M, N, K, split, epi, bt):
    A = _r(M, K, seed=1)
    B = _r(N, K, seed=2, scale=K ** -0.5)          # weight (N, K): B operand rows (bt: stored (K, N))
    Ad = A.float().to(DEV)
    Bd = (B.t() if bt else B).contiguous().float().to(DEV)
    ref = A @ B.t()
    kw = {}
    if epi == "bias_relu_resid":
        bias, resid = _r(N, seed=4), _r(M, N, seed=5)
        kw = dict(bias=bias.float().to(DEV), resid=resid.float().to(DEV), relu=1)
        ref = torch.relu(ref + bias + resid)

    def b_fn():
        b = _rows(Bd)
        b.trans = int(bt)
        return b
    _check(ref, M, N, K, lambda: _rows(Ad), b_fn, split, **kw)


def test_split_conv_gemm_fp32_accuracy():
    """Implicit dilated conv (3 taps, dilation 4, zero outside each video; ragged lengths 4096 + 2900)."""
    Ts, cin, N, dil = (4096, 2900), 256, 256, 4
    M, K = sum(Ts), 3 * cin
    X = _r(M, cin, seed=11)
    W = _r(N, K, seed=12, scale=K ** -0.5)          # [n][tap * cin + c]
    Xd, Wd = X.float().to(DEV), W.float().to(DEV)
    offs = [0, Ts[0], M]
    import ctypes
    off_host = (ctypes.c_int * 3)(*offs)

    def a_fn():
        a = _rows(Xd, cin)
        a.conv_taps, a.conv_cin, a.conv_dil, a.seq_len = 3, cin, dil, Ts[0]
        a.seq_off, a.nseq = ctypes.addressof(off_host), 2
        return a
    cols = []
    for tap in range(3):
        s = (tap - 1) * dil
        sh = torch.zeros_like(X)
        for v in range(2):
            lo, hi = offs[v], offs[v + 1]
            xv = X[lo:hi]
            if s >= 0:
                sh[lo:hi - s] = xv[s:]
            else:
                sh[lo - s:hi] = xv[:hi - lo + s]
        cols.append(sh)
    ref = torch.cat(cols, 1) @ W.t()
    _check(ref, M, N, K, a_fn, lambda: _rows(Wd))


def test_split_concat_operand_fp32_accuracy():
    """A = [Y | F] concatenated at k = 512 (the X2Y Y_W GEMM's operand), K = 1024."""
    M, N = 8192, 256
    Y, F = _r(M, 512, seed=21), _r(M, 512, seed=22)
    W = _r(N, 1024, seed=23, scale=1024 ** -0.5)
    Yd, Fd, Wd = Y.float().to(DEV), F.float().to(DEV), W.float().to(DEV)

    def a_fn():
        a = _rows(Yd)
        a.ptr1, a.ld1, a.k_split = nx.ptr(Fd), 512, 512
        return a
    _check(torch.cat([Y, F], 1) @ W.t(), M, N, 1024, a_fn, lambda: _rows(Wd))


def test_split_mode_north_star_step_vs_oracle(monkeypatch):
    """The bench's north-star step (FACT_CLIP, HAViD holdout dims, T=4096, 2 videos, lockstep) with
    every eligible frame-level GEMM in FX_PREC_F32S, against the fp64 oracle at the fp32 path's own
    parity bounds: TDU segments identical, predictions identical, per-frame logits within 1e-3, loss
    within 1e-4 relative, every gradient within 2e-3."""
    import bench
    from helpers import GruKinks, compare_grads, oracle_batch
    from oracle import fact_oracle as fo
    from test_gpu_backward import _check_forward, _gpu_step, _segments
    cfg = bench.make_cfg()
    T, D, C = 4096, 2048, 75
    net, text = bench.build_model(cfg, D, C, device=DEV, seed=0)
    net.train()
    vids = [bench.make_video(T, D, C, cfg, seed=s) for s in (1, 2)]
    kinks = GruKinks(monkeypatch)
    from factmx.dp import DataParallel
    dp = DataParallel(net)
    with fxf.gemm_precision("fp32s"):
        loss, saves = _gpu_step(net, vids, dp=dp)
    S = _segments(net)
    spec = fo.resolve_spec(cfg, D, C, clip=True)
    ref_loss, ref_grads, outs = oracle_batch(spec, net, vids, text)
    assert S == [[len(r["tdu"].starts) for r in o["blocks"] if r["type"] == "U"] for o in outs], S
    _check_forward(net, spec, outs, saves, text)
    assert abs(loss - ref_loss) <= 1e-4 * abs(ref_loss), (loss, ref_loss)
    compare_grads(net, ref_grads, rtol=2e-3, relaxed=kinks.flipped_prefixes(len(vids)), what="fp32s T=4096: ")
