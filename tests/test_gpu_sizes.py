"""Workspace reservations across video lengths (GPU).

Every entry point sizes its split-K slabs from the same split heuristics its GEMMs use, and a
GEMM whose slabs would leave the reservation fails loudly (WsBound) instead of overrunning.  The
split factors depend on the row count (tile counts, 64-deep stages, the side stream's deferred
split), so a length the parity tests do not hit can still pick a bigger split for one piece than
the reservation assumed (it did: 1724 rows, the x2y dW_y piece).  This sweep runs a full training
step of the benchmark model (HAViD-holdout dims) at single lengths and ragged pairs spread over
1..8192 rows -- both the lockstep path and the data-parallel flat-gradient path -- and requires
a finite loss and finite gradients; parity at chosen lengths is test_gpu_backward's job.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

LENGTHS = [(2,), (63,), (65,), (200,), (511,), (777,), (1000,), (1724,), (2047,), (2500,), (3333,), (4097,),
           (6000,), (8192,), (100, 1624), (700, 1024), (1500, 2999), (4096, 4095), (33, 5000)]


@pytest.fixture(scope="module")
def model():
    import bench
    cfg = bench.make_cfg()
    net, _ = bench.build_model(cfg, 2048, 75, device=DEV, seed=0)
    net.train()
    return bench, cfg, net


@pytest.mark.parametrize("Ts", LENGTHS, ids=["+".join(map(str, t)) for t in LENGTHS])
def test_training_step_lengths(Ts, model):
    bench, cfg, net = model
    from factmx.dp import DataParallel
    vids = [bench.make_video(T, 2048, 75, cfg, seed=40 + i, nseg=max(1, min(10, T // 8))) for i, T in enumerate(Ts)]
    dp = DataParallel(net)
    dp.zero_grad()
    loss, _ = net([torch.from_numpy(f).to(DEV) for f, _ in vids], [torch.from_numpy(l_).to(DEV) for _, l_ in vids],
                  compute_loss=True)
    loss.backward()
    dp.finish_gradients()
    torch.cuda.synchronize()
    assert np.isfinite(loss.item()), (Ts, loss.item())
    bad = [n for n, p in net.named_parameters() if p.grad is None or not torch.isfinite(p.grad).all()]
    assert not bad, (Ts, bad[:5])
