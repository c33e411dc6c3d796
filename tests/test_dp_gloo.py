"""Data parallelism over whole videos (factmx.dp.FlatGradReducer), world_size 2 on gloo/CPU.

The reference averages per-video losses over its batch (blocks.py:913-915), so
sharding videos over ranks and all-reducing the mean of the gradients must equal
the single-process gradient of the batch-mean loss.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from factmx.dp import FlatGradReducer


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(12, 16), torch.nn.ReLU(), torch.nn.Linear(16, 5))


def _videos():
    g = torch.Generator().manual_seed(1)
    return [torch.randn(7 + 3 * i, 12, generator=g) for i in range(4)]


def _video_loss(net, x):
    return net(x).pow(2).mean()


def _worker(rank, world, port, out_path, bucket_mb):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = _model()
        red = FlatGradReducer(net.parameters(), bucket_mb=bucket_mb)
        vids = _videos()
        mine = vids[rank::world]
        for step in range(2):   # two steps: zero_grad must keep the views and reset them
            red.zero_grad()
            loss = sum(_video_loss(net, x) for x in mine) / len(mine)
            loss.backward()
            red.all_reduce_mean()
            for p in net.parameters():   # backward accumulated into the flat buffer itself
                assert red.flat.data_ptr() <= p.grad.data_ptr() < red.flat.data_ptr() + red.flat.numel() * 4
        if rank == 0:
            torch.save({n: p.grad.clone() for n, p in net.named_parameters()}, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bucket_mb", [64, 0.0005])   # one bucket / many tiny buckets
def test_dp_mean_grads_equal_single_process(tmp_path, bucket_mb):
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), out, bucket_mb), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    net = _model()
    vids = _videos()
    loss = sum(_video_loss(net, x) for x in vids) / len(vids)
    loss.backward()
    for n, p in net.named_parameters():
        torch.testing.assert_close(got[n], p.grad, rtol=1e-5, atol=1e-7)


def test_zero_grad_detects_detached_views():
    net = _model()
    red = FlatGradReducer(net.parameters())
    next(net.parameters()).grad = None
    with pytest.raises(RuntimeError):
        red.zero_grad()


def test_single_process_reduce_is_noop():
    net = _model()
    red = FlatGradReducer(net.parameters())
    red.flat.fill_(3.0)
    red.all_reduce_mean()
    assert torch.all(red.flat == 3.0)
