"""BiGRU timeouts are reported, not silent (GPU).

The persistent BiGRU kernel (gru.hip) spreads each direction over 16 workgroups that exchange the
hidden state through L2 with bounded spins; a workgroup that gives up on a peer ends the launch and
sets the caller's status word (FX_STATUS_GRU_TIMEOUT).  Forcing a tiny spin bound must surface as
FactmxNativeError at the step's single host read-back -- resolved at the first read of the saves or
at the end of the backward pass -- and the next normal step must succeed.
"""
import pytest
import torch

from helpers import load_fixture, tiny_meta, cfg_from_meta, tiny_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_gru_timeout_raises_at_readback(monkeypatch):
    import paramgen as pg
    from factmx import functional as fxf
    from factmx import native as nx
    from factmx.models.blocks import FACT_CLIP
    from factmx.models.loss import MatchCriterion
    fx = load_fixture("tiny_clip_iid")          # many TDU segments: long GRU sequences
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    feats, label, text = tiny_inputs(meta)
    net = FACT_CLIP(cfg, meta["D"], meta["C"], text_embeddings=torch.from_numpy(text).float())
    with torch.no_grad():
        for n, p in net.named_parameters():
            p.copy_(torch.from_numpy(pg.param_value(n, p.shape, meta["seed"])))
    net.mcriterion = MatchCriterion(cfg, meta["C"], [])
    net = net.to(DEV).train()
    seqs = [torch.from_numpy(feats).float().to(DEV)] * 2
    labs = [torch.from_numpy(label).to(DEV)] * 2
    monkeypatch.setattr(fxf, "GRU_SPIN_MAX", 1)      # give up after two empty polls
    with pytest.raises(nx.FactmxNativeError, match="GRU"):
        loss, saves = net(seqs, labs, compute_loss=True)
        saves[0]["pred"]        # the step's read-back resolves here (or at the end of backward)
    torch.cuda.synchronize()
    monkeypatch.setattr(fxf, "GRU_SPIN_MAX", 1)
    with pytest.raises(nx.FactmxNativeError, match="GRU"):
        loss, _ = net(seqs, labs, compute_loss=True)
        loss.backward()         # ... resolved by the autograd callback at the end of the backward pass
    torch.cuda.synchronize()
    monkeypatch.setattr(fxf, "GRU_SPIN_MAX", 0)
    loss, _ = net(seqs, labs, compute_loss=True)
    loss.backward()
    fxf.check_device_status()
    assert torch.isfinite(loss).item()


def test_gru_backward_timeout_raises_and_skips_adam(monkeypatch):
    """A BiGRU timeout in the BACKWARD pass only (the forward ran normally): the status word is copied
    after the backward's kernels, FusedAdam's update on the invalid gradients is skipped on the device
    (parameters and moments unchanged), and the failure is raised at the next forward, naming the
    backward pass; the step after that trains normally."""
    import paramgen as pg
    from factmx import functional as fxf
    from factmx import native as nx
    from factmx.dp import DataParallel
    from factmx.models.blocks import FACT_CLIP
    from factmx.models.loss import MatchCriterion
    from factmx.optim import FusedAdam
    fx = load_fixture("tiny_clip_iid")
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    feats, label, text = tiny_inputs(meta)
    net = FACT_CLIP(cfg, meta["D"], meta["C"], text_embeddings=torch.from_numpy(text).float())
    with torch.no_grad():
        for n, p in net.named_parameters():
            p.copy_(torch.from_numpy(pg.param_value(n, p.shape, meta["seed"])))
    net.mcriterion = MatchCriterion(cfg, meta["C"], [])
    net = net.to(DEV).train()
    dp = DataParallel(net)
    opt = FusedAdam(net.parameters(), lr=1e-3, max_grad_norm=10.0, grad_flat=dp.flat)
    seqs = [torch.from_numpy(feats).float().to(DEV)] * 2
    labs = [torch.from_numpy(label).to(DEV)] * 2
    monkeypatch.setattr(fxf, "GRU_SPIN_MAX", 0)
    dp.zero_grad()
    loss, saves = net(seqs, labs, compute_loss=True)
    saves[0]["pred"]                           # the forward's own read-back: clean
    monkeypatch.setattr(fxf, "GRU_SPIN_MAX", 1)   # only the backward's GRU gives up
    loss.backward()
    w0, m0 = opt.flat.clone(), opt.exp_avg.clone()
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(opt.flat, w0) and torch.equal(opt.exp_avg, m0), "Adam applied invalid gradients"
    monkeypatch.setattr(fxf, "GRU_SPIN_MAX", 0)
    with pytest.raises(nx.FactmxNativeError, match="BACKWARD"):
        net(seqs, labs, compute_loss=True)
    dp.zero_grad()
    loss, _ = net(seqs, labs, compute_loss=True)
    loss.backward()
    opt.step()
    fxf.check_device_status()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item() and not torch.equal(opt.flat, w0)
