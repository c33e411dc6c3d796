"""Grid-barrier timeouts of the two persistent kernels report through the device status word and leave
the library usable (GPU).

* the token kernel (tokdec.hip, every SCA / SA decoder layer's token rows): a tiny poll bound
  (fx_debug_set_spin(0, 1)) makes workgroups give up at a grid barrier -> FX_STATUS_TOK_TIMEOUT in the
  status word and check_device_status() raises; then, with the default bound back, more decoder calls than
  the kernel's 512 round-robin barrier slots (so the slot of the timed-out launch is dealt again) give
  outputs bitwise equal to the run before the timeout;
* the one-launch X2Y f2a backward core (x2y_core.hip x2y_f2a_bwd_kernel<3>, the default for >= 64 key
  chunks): the same with fx_debug_set_spin(1, 1) -> FX_STATUS_X2Y_TIMEOUT, then bitwise-equal gradients.
The reference has no counterpart (its attention is torch.nn.MultiheadAttention, basic.py:396-523, 349-389):
these are the failure paths of this library's own barriers."""
import math

import pytest
import torch

from factmx import functional as fxf
from factmx import native as nx
from factmx.models import basic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _status():
    torch.cuda.synchronize()
    return int(fxf.device_status(torch.device(DEV))[0].item())


def _clear_status():
    fxf.device_status(torch.device(DEV)).zero_()
    fxf._bwd_status.clear()
    torch.cuda.synchronize()


def _spin(which, polls):
    assert nx.load().fx_debug_set_spin(which, polls) == 0


def test_token_kernel_timeout_sets_status_and_slot_reuse_is_clean():
    torch.manual_seed(0)
    layer = basic.SALayer(256, 8, dim_feedforward=512, dropout=0.0, attn_dropout=0.0)
    dec = basic.SADecoder(256, 256, 512, layer, 2, in_map=False).to(DEV)
    assert basic._fused_decoder_ok(dec)
    x = torch.randn(32, 1, 256, device=DEV)      # (<= 32 tokens per video: the token kernel's shapes)
    qp = torch.randn(32, 1, 256, device=DEV)
    _clear_status()
    with torch.no_grad():
        ref = dec(x, qp).clone()
    assert _status() == 0
    try:
        _spin(0, 1)
        hit = 0
        with torch.no_grad():
            for _ in range(8):
                dec(x, qp)
                hit |= _status()
                if hit & nx.STATUS_TOK_TIMEOUT:
                    break
    finally:
        _spin(0, 0)
    assert hit & nx.STATUS_TOK_TIMEOUT, hit
    with pytest.raises(nx.FactmxNativeError, match="FX_STATUS_TOK_TIMEOUT"):
        fxf.check_device_status(torch.device(DEV))
    assert _status() == 0
    # more launches than the 512 barrier slots of the stream: every slot, the timed-out one included,
    # is dealt again; each must start re-armed
    with torch.no_grad():
        for i in range(300):
            y = dec(x, qp)
            if i % 50 == 49:
                assert torch.equal(y, ref), f"call {i}: token-kernel output differs after a timed-out launch"
    assert torch.equal(y, ref)
    assert _status() == 0


def _x2y_case():
    g = torch.Generator().manual_seed(11)
    H, xdim, ydim, outdim, nq = 512, 256, 256, 192, 32
    Ts = (4096, 300)       # 64 + 5 key chunks: the one-launch fused f2a backward
    X = torch.randn(sum(Ts), xdim, generator=g).to(DEV).requires_grad_(True)
    Y = torch.randn(nq * len(Ts), ydim, generator=g).to(DEV).requires_grad_(True)
    W = {}
    for n, shp in (("wk", (H, xdim)), ("bk", (H,)), ("wv", (H, xdim)), ("bv", (H,)), ("wq", (H, ydim)),
                   ("bq", (H,)), ("wy", (outdim, ydim + H)), ("by", (outdim,))):
        W[n] = (torch.randn(*shp, generator=g) / math.sqrt(shp[-1])).to(DEV).requires_grad_(True)
    rows = ([0, Ts[0], sum(Ts)], [0, nq, 2 * nq])
    gout = torch.randn(nq * len(Ts), outdim, generator=g).to(DEV)
    glog = torch.randn(nq * sum(Ts), generator=g).to(DEV)
    return X, Y, W, rows, gout, glog


def _x2y_step(X, Y, W, rows, gout, glog):
    for t in [X, Y] + list(W.values()):
        t.grad = None
    out, logit, _ = fxf.X2YFn.apply(X, Y, None, None, rows, W["wk"], W["bk"], W["wv"], W["bv"], W["wq"], W["bq"],
                                    W["wy"], W["by"], 0.0, 0)
    ((out * gout).sum() + (logit.reshape(-1) * glog).sum()).backward()
    torch.cuda.synchronize()
    return [X.grad.clone(), Y.grad.clone()] + [W[n].grad.clone() for n in sorted(W)]


def test_x2y_f2a_backward_timeout_sets_status_then_clean():
    case = _x2y_case()
    _clear_status()
    ref = _x2y_step(*case)
    assert _status() == 0
    try:
        _spin(1, 1)
        hit = 0
        for _ in range(8):
            _x2y_step(*case)
            hit |= _status()
            if hit & nx.STATUS_X2Y_TIMEOUT:
                break
    finally:
        _spin(1, 0)
    assert hit & nx.STATUS_X2Y_TIMEOUT, hit
    with pytest.raises(nx.FactmxNativeError, match="FX_STATUS_X2Y_TIMEOUT"):
        fxf.check_device_status(torch.device(DEV))
    assert _status() == 0
    for _ in range(3):
        got = _x2y_step(*case)
    for a, b in zip(got, ref):
        assert torch.equal(a, b), "f2a backward gradients differ after a timed-out launch"
    assert _status() == 0
