"""Whole-decoder kernel path (fx_decoder_fwd/bwd) vs the float64 oracle restatement of
SCADecoder / SADecoder (basic.py:525-593; oracle/fact_oracle.py sca_decoder / sa_decoder):
outputs and the gradients of every parameter, the token input, the query positions
(action_query), the frame memory and the frame positions (GPU)."""
import pytest
import torch

from factmx.models import basic
from oracle import fact_oracle as fo

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _seed_params(mod, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for n, p in mod.named_parameters():
            p.copy_(torch.randn(p.shape, generator=g) * (0.5 if "norm" in n else p.shape[-1] ** -0.5) +
                    (1.0 if n.endswith("norm1.weight") or n.endswith("norm2.weight") or n.endswith("norm3.weight")
                     or n == "norm.weight" else 0.0))


def _close(a, b, tol, what):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item()
    assert err <= tol * max(ref, 1e-3), f"{what}: max err {err:.3e} vs ref max {ref:.3e}"


@pytest.mark.parametrize("R,A,h,FF,Hm,L,T,use_pos,use_qpos", [
    (32, 256, 8, 512, 512, 6, 1024, False, True),     # HAViD input-block dims (T shortened)
    (8, 32, 4, 64, 64, 2, 200, True, True),           # tiny config; Hm == A -> packed in_proj weight
    (5, 48, 6, 40, 72, 3, 77, True, False),           # ragged sizes, no query positions
])
def test_sca_decoder_vs_oracle(R, A, h, FF, Hm, L, T, use_pos, use_qpos):
    layer = basic.SCALayer(A, Hm, h, FF, dropout=0.0, attn_dropout=0.0)
    dec = basic.SCADecoder(A, A, 2 * A, layer, L, norm=torch.nn.LayerNorm(A), in_map=False)
    _seed_params(dec, 1)
    dec = dec.to(DEV).train()
    g = torch.Generator().manual_seed(2)
    tgt = torch.randn(R, 1, A, generator=g, dtype=torch.float64)
    mem = torch.randn(T, 1, Hm, generator=g, dtype=torch.float64)
    pos = torch.randn(T, 1, Hm, generator=g, dtype=torch.float64) if use_pos else None
    qpos = torch.randn(R, 1, A, generator=g, dtype=torch.float64) if use_qpos else None
    gout = torch.randn(R, 2 * A, generator=g, dtype=torch.float64)

    def dev(t):
        return None if t is None else t.float().to(DEV).requires_grad_(True)
    tg, mm, ps, qp = dev(tgt), dev(mem), dev(pos), dev(qpos)
    out = dec(tg, mm, pos=ps, query_pos=qp)
    (out[:, 0] * gout.float().to(DEV)).sum().backward()
    P = {n: p.detach().double().cpu().requires_grad_(True) for n, p in dec.named_parameters()}
    rt, rm = tgt.clone().requires_grad_(True), mem.clone().requires_grad_(True)
    rp = None if pos is None else pos.clone().requires_grad_(True)
    rq = None if qpos is None else qpos.clone().requires_grad_(True)
    ref = fo.sca_decoder(P, "", rt[:, 0], rm[:, 0], None if rp is None else rp[:, 0],
                         None if rq is None else rq[:, 0], L, h)
    (ref * gout).sum().backward()
    _close(out[:, 0], ref, 2e-5, "out")
    _close(tg.grad[:, 0], rt.grad[:, 0], 1e-4, "d tgt")
    _close(mm.grad[:, 0], rm.grad[:, 0], 1e-4, "d memory")
    if rp is not None:
        _close(ps.grad[:, 0], rp.grad[:, 0], 1e-4, "d pos")
    if rq is not None:
        _close(qp.grad[:, 0], rq.grad[:, 0], 1e-4, "d query_pos")
    for n, p in dec.named_parameters():
        _close(p.grad, P[n].grad, 2e-4, f"d {n}")


@pytest.mark.parametrize("R,A,h,FF,L", [(32, 256, 8, 512, 1), (8, 32, 4, 64, 3)])
def test_sa_decoder_vs_oracle(R, A, h, FF, L):
    layer = basic.SALayer(A, h, dim_feedforward=FF, dropout=0.0, attn_dropout=0.0)
    dec = basic.SADecoder(A, A, 2 * A, layer, L, in_map=False)
    _seed_params(dec, 3)
    dec = dec.to(DEV).train()
    g = torch.Generator().manual_seed(4)
    tgt = torch.randn(R, 1, A, generator=g, dtype=torch.float64)
    qpos = torch.randn(R, 1, A, generator=g, dtype=torch.float64)
    gout = torch.randn(R, 2 * A, generator=g, dtype=torch.float64)
    tg = tgt.float().to(DEV).requires_grad_(True)
    qp = qpos.float().to(DEV).requires_grad_(True)
    out = dec(tg, qp)
    (out[:, 0] * gout.float().to(DEV)).sum().backward()
    P = {n: p.detach().double().cpu().requires_grad_(True) for n, p in dec.named_parameters()}
    rt, rq = tgt.clone().requires_grad_(True), qpos.clone().requires_grad_(True)
    ref = fo.sa_decoder(P, "", rt[:, 0], rq[:, 0], L, h)
    (ref * gout).sum().backward()
    _close(out[:, 0], ref, 2e-5, "out")
    _close(tg.grad[:, 0], rt.grad[:, 0], 1e-4, "d tgt")
    _close(qp.grad[:, 0], rq.grad[:, 0], 1e-4, "d query_pos")
    for n, p in dec.named_parameters():
        _close(p.grad, P[n].grad, 2e-4, f"d {n}")


def test_fused_path_is_taken():
    layer = basic.SALayer(32, 4, dim_feedforward=64, dropout=0.0, attn_dropout=0.0)
    dec = basic.SADecoder(32, 32, 64, layer, 1, in_map=False).to(DEV)
    assert basic._fused_decoder_ok(dec)
    dec(torch.randn(8, 1, 32, device=DEV), torch.randn(8, 1, 32, device=DEV))
    assert hasattr(dec, "_fx_spec")


@pytest.mark.parametrize("M,N,K,amode,btrans", [(64, 256, 256, 0, 0), (64, 512, 256, 1, 0), (32, 256, 768, 0, 1),
                                                 (37, 80, 256, 1, 0), (64, 256, 76, 0, 1)])
def test_token_kernel_gemm_phase(M, N, K, amode, btrans):
    """One GEMM phase of the persistent token kernel (tokdec.hip) vs float64 torch: plain or LayerNorm-staged
    A rows, W or W^T, bias + residual epilogue."""
    from factmx import functional as fxf
    from factmx import native as nx
    g = torch.Generator().manual_seed(5)
    a = torch.randn(M, K, generator=g, dtype=torch.float64)
    w = torch.randn(K, N, generator=g, dtype=torch.float64) if btrans else torch.randn(N, K, generator=g, dtype=torch.float64)
    w = w / K ** 0.5
    lw, lb = 1 + 0.3 * torch.randn(K, generator=g, dtype=torch.float64), 0.2 * torch.randn(K, generator=g, dtype=torch.float64)
    bias, res = torch.randn(N, generator=g, dtype=torch.float64), torch.randn(M, N, generator=g, dtype=torch.float64)
    d = [t.float().to(DEV).contiguous() for t in (a, w, lw, lb, bias, res)]
    c = torch.empty(M, N, device=DEV)
    st = fxf.device_status(c.device)
    lib = nx.load()
    assert lib.fx_tok_gemm(nx.ptr(d[0]), K, M, N, K, amode, nx.ptr(d[2]), nx.ptr(d[3]), nx.ptr(d[1]), N if btrans else K,
                           btrans, nx.ptr(d[4]), nx.ptr(d[5]), N, nx.ptr(c), N, nx.ptr(st), nx.stream()) == 0
    torch.cuda.synchronize()
    assert int(st[0]) == 0
    x = fo.layer_norm(a, lw, lb) if amode else a
    ref = x @ (w if btrans else w.t()) + bias + res
    _close(c, ref, 2e-5, "c")
