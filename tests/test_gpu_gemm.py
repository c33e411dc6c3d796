"""fx_gemm across both kernels (64x64 LDS-tiled / direct small-shape) and every epilogue option,
vs float64 torch on the same inputs (GPU).  Shapes are picked so the automatic path choice
exercises: direct (token rows, shallow K, few tiles, batched heads, cross-block split-K with the
fused last-block reduction) and tiled (with and without split-K)."""
import pytest
import torch

from factmx import functional as fxf
from factmx import native as nx

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g, dtype=torch.float64) * scale


def _operand(t2d_or_3d, trans, batch_stride=0):
    o = nx.Operand()
    o.ptr = nx.ptr(t2d_or_3d)
    o.ld = t2d_or_3d.shape[-1]
    o.trans = int(trans)
    o.conv_dir = 1
    o.batch_stride = batch_stride
    return o


CASES = [
    # M, N, K, batch, a_trans, b_trans, split
    (32, 512, 512, 1, False, False, 1),     # token projection (direct)
    (32, 256, 1024, 1, False, True, 4),     # token dX (direct, split-K)
    (256, 257, 32, 1, True, True, 1),       # token dW, K = Nact (direct)
    (256, 257, 4096, 1, True, True, 13),    # frame-level dW, few tiles (direct, split-K)
    (4096, 32, 32, 8, True, True, 1),       # per-head attention products (direct, batched)
    (32, 32, 4096, 8, False, True, 32),     # per-head dK/dV-like (direct, batched split-K)
    (96, 200, 1000, 1, False, False, 1),    # ragged edges (direct)
    (7, 5, 3, 1, False, True, 1),           # tiny
    (600, 520, 300, 1, False, False, 1),    # tiled
    (600, 520, 3000, 1, True, False, 6),    # tiled split-K, fused reduction
    (1000, 700, 77, 2, False, True, 1),     # tiled, batched, ragged
    (600, 520, 3001, 1, True, True, 6),     # weight gradient, K tail (COLS_KT: rows past K read as zero)
    (512, 513, 6996, 1, True, True, 13),    # the shipped yaml's ragged 4096 + 2900 rows (K tail, wide tile)
    (640, 256, 1000, 2, True, True, 1),     # K tail, batched
]


@pytest.mark.parametrize("M,N,K,batch,at,bt,split", CASES)
@pytest.mark.parametrize("epi", ["plain", "bias_relu_resid", "beta_gate"])
def test_gemm(M, N, K, batch, at, bt, split, epi):
    A = _r(batch, M, K, seed=1)
    B = _r(batch, K, N, seed=2, scale=K ** -0.5)
    Ad = (A.transpose(1, 2) if at else A).contiguous().float().to(DEV)
    Bd = (B if bt else B.transpose(1, 2)).contiguous().float().to(DEV)
    a = _operand(Ad, at, Ad[0].numel())
    b = _operand(Bd, bt, Bd[0].numel())
    ref = A @ B
    c0 = _r(batch, M, N, seed=3)
    c = c0.float().to(DEV).contiguous()
    kw = {}
    if epi == "bias_relu_resid" and batch == 1:
        bias, resid = _r(N, seed=4), _r(M, N, seed=5)
        kw = dict(bias=bias.float().to(DEV), resid=resid.float().to(DEV), relu=1)
        ref = torch.relu(ref + bias + resid)
    elif epi == "beta_gate" and batch == 1:
        gate = _r(M, N, seed=6)
        kw = dict(beta=0.5, gate=gate.float().to(DEV))
        ref = torch.where(gate > 0, ref + 0.5 * c0, torch.zeros_like(ref))
    elif epi != "plain":
        pytest.skip("epilogue operands are single-batch")
    fxf.gemm(M, N, K, a, b, c, N, split=split, batch=batch, c_bs=M * N, **kw)
    torch.cuda.synchronize()
    err = (c.double().cpu() - ref).abs().max().item()
    assert err <= 1e-5 * (1 + ref.abs().max().item()) + 1e-6 * K ** 0.5, err


@pytest.mark.parametrize("M,K,split", [(256, 32, 1), (256, 4096, 13), (512, 4096, 5), (512, 6996, 13), (256, 2900, 1)])
def test_gemm_fused_bias_column(M, K, split):
    """dW|db in one GEMM: the B operand's last column is a virtual ones column (c_last gets row sums)."""
    N1 = 200
    dy = _r(K, M, seed=7)         # (rows, out)
    x = _r(K, N1, seed=8)         # (rows, in)
    dyd, xd = dy.float().to(DEV), x.float().to(DEV)
    dw = _r(M, N1, seed=9)
    db = _r(M, seed=10)
    dwd, dbd = dw.float().to(DEV).contiguous(), db.float().to(DEV).contiguous()
    b = _operand(xd, True)
    b.ones_col = N1 + 1
    fxf.gemm(M, N1 + 1, K, _operand(dyd, True), b, dwd, N1, beta=1.0, split=split, c_last=dbd)
    torch.cuda.synchronize()
    # fp32 accumulation over K terms of unit-variance products: rounding grows ~sqrt(K) (the 128x64
    # tile runs one serial MFMA chain per split instead of two k-halves, so ~1.4x the 64x64 error).
    atol = max(1e-4, 5e-6 * K ** 0.5)
    torch.testing.assert_close(dwd.double().cpu(), dw + dy.t() @ x, rtol=1e-5, atol=atol)
    torch.testing.assert_close(dbd.double().cpu(), db + dy.sum(0), rtol=1e-5, atol=atol)


def test_split_k_repeat_is_deterministic():
    """The per-tile arrival counters re-arm: back-to-back split-K launches give identical bits."""
    A = _r(3000, 64, seed=11).float().to(DEV)
    B = _r(3000, 96, seed=12).float().to(DEV)
    outs = []
    for _ in range(3):
        c = torch.empty(64, 96, device=DEV)
        fxf.gemm(64, 96, 3000, _operand(A, True), _operand(B, True), c, 96, split=8)
        outs.append(c)
    for _ in range(3):
        c = torch.empty(64, 96, device=DEV)
        fxf.gemm(64, 96, 3000, _operand(A, True), _operand(B, True), c, 96, split=3)
        outs.append(c)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    assert torch.equal(outs[3], outs[4])
    torch.testing.assert_close(outs[0], outs[3], rtol=1e-5, atol=1e-4)
