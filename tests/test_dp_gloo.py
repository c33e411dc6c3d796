"""Data parallelism over whole videos (factmx.dp), world_size 2 on gloo/CPU.

The reference averages per-video losses over its batch (blocks.py:913-915), so
sharding videos over ranks and all-reducing the mean of the gradients must equal
the single-process gradient of the batch-mean loss.  DataParallel additionally
broadcasts rank 0's weights, launches each block's bucket from a backward hook
(overlapping the rest of backward) and the rank-sharded DataLoader hands every
rank its share of the same global batch.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from factmx.dp import DataParallel, FlatGradReducer, mark_block_input, mark_block_part


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


class _ToyBlocks(torch.nn.Module):
    """block_list + a parameter shared by every block (like FACT's action queries)."""

    def __init__(self, seed=0):
        super().__init__()
        torch.manual_seed(seed)
        self.q = torch.nn.Parameter(torch.randn(12) * 0.1)
        self.block_list = torch.nn.ModuleList([torch.nn.Linear(12, 12), torch.nn.Linear(12, 12),
                                               torch.nn.Linear(12, 5)])

    def forward(self, x):
        h = x
        for k, b in enumerate(self.block_list):
            mark_block_input(self, k, h)
            h = torch.tanh(b(h + (self.q if h.shape[-1] == 12 else 0)))
        return h


def _dp_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = _ToyBlocks(seed=rank)          # rank 1 starts from other weights: the broadcast fixes that
        dp = DataParallel(net, bucket_mb=0.0002)
        vids = _videos()
        mine = vids[rank::world]
        for step in range(2):
            dp.zero_grad()
            loss = sum(net(x).pow(2).mean() for x in mine) / len(mine)   # per-video forwards
            loss.backward()
            early = list(dp.hook_launched)
            dp.finish_gradients()
        if rank == 0:
            torch.save({"grads": {n: p.grad.clone() for n, p in net.named_parameters()},
                        "early": torch.tensor(early)}, out_path)
    finally:
        dist.destroy_process_group()


def test_data_parallel_hooks_broadcast_and_mean(tmp_path):
    out = str(tmp_path / "dp.pt")
    mp.spawn(_dp_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    # blocks 2 and 1 launched from backward hooks, in backward order; block 0 (input needs no grad)
    # and the shared parameter at finish_gradients
    assert got["early"].tolist() == [2, 1]
    net = _ToyBlocks(seed=0)
    vids = _videos()
    loss = sum(net(x).pow(2).mean() for x in vids) / len(vids)
    loss.backward()
    for n, p in net.named_parameters():
        torch.testing.assert_close(got["grads"][n], p.grad, rtol=1e-5, atol=1e-7)


class _ToyInputBlock(torch.nn.Module):
    """A first block whose input is the data: part `b` reads only the output of part `a`
    (InputBlock: the action branch reads the frame branch's output)."""
    dp_parts = ("b",)

    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(12, 12)
        self.b = torch.nn.Linear(12, 12)

    def forward(self, h):
        f = torch.tanh(self.a(h))
        ctx = self.__dict__.get("_dp_ctx")
        if ctx is not None:
            mark_block_part(ctx[0], ctx[1], "b", f)
        return torch.tanh(self.b(f)) + f


class _ToyParts(torch.nn.Module):
    """_ToyBlocks with a first block split in two parts and a head applied after the last block (the
    CLIP projection), registered BEFORE the blocks so its slice is not adjacent to theirs."""
    dp_head_modules = ("head",)

    def __init__(self, seed=0):
        super().__init__()
        torch.manual_seed(seed)
        self.q = torch.nn.Parameter(torch.randn(12) * 0.1)
        self.head = torch.nn.Linear(5, 3)
        self.block_list = torch.nn.ModuleList([_ToyInputBlock(), torch.nn.Linear(12, 12), torch.nn.Linear(12, 5)])

    def forward(self, x):
        h = x
        for k, b in enumerate(self.block_list):
            mark_block_input(self, k, h)
            b.__dict__["_dp_ctx"] = (self, k)
            h = torch.tanh(b(h + (self.q if h.shape[-1] == 12 else 0)))
        return self.head(h)


def _parts_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = _ToyParts(seed=rank)
        dp = DataParallel(net, bucket_mb=0.0002)
        mine = _videos()[rank::world]
        for step in range(2):
            dp.zero_grad()
            loss = sum(net(x).pow(2).mean() for x in mine) / len(mine)
            issued = []
            orig = dp._issue
            dp._issue = lambda bs, orig=orig: (issued.append(sum(b.numel() for b in bs)), orig(bs))[1]
            loss.backward()
            early = [str(k) for k in dp.hook_launched]
            dp.finish_gradients()
            dp._issue = orig
        if rank == 0:
            torch.save({"grads": {n: p.grad.clone() for n, p in net.named_parameters()}, "early": early,
                        "issued": issued, "tail": dp.tail_bytes}, out_path)
    finally:
        dist.destroy_process_group()


def test_data_parallel_part_and_head_buckets(tmp_path):
    out = str(tmp_path / "dpp.pt")
    mp.spawn(_parts_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    # hooks in backward order: block 2, block 1, then block 0's part b from the hook on part a's output
    assert got["early"] == ["2", "1", "(0, 'b')"]
    # the head (5x3 + 3) goes out with the first hook, before block 2's bucket
    assert got["issued"][0] == 5 * 3 + 3 and got["issued"][1] == 12 * 5 + 5
    # left for finish_gradients: block 0's part a and the shared queries only (+ the status word: none
    # on gloo/CPU)
    assert got["tail"] == 4 * ((12 * 12 + 12) + 12)
    net = _ToyParts(seed=0)
    vids = _videos()
    (sum(net(x).pow(2).mean() for x in vids) / len(vids)).backward()
    for n, p in net.named_parameters():
        torch.testing.assert_close(got["grads"][n], p.grad, rtol=1e-5, atol=1e-7)


def _accum_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = _ToyBlocks(seed=0)
        dp = DataParallel(net, bucket_mb=0.0002)
        x = _videos()[rank]
        dp.zero_grad()
        net(x).pow(2).mean().backward()
        raised = False
        try:             # a second forward before zero_grad: its hooks would add unreduced gradients
            net(x).pow(2).mean().backward()
        except RuntimeError:
            raised = True
        dp.finish_gradients()
        if rank == 0:
            torch.save(torch.tensor([raised]), out_path)
    finally:
        dist.destroy_process_group()


def test_data_parallel_refuses_gradient_accumulation(tmp_path):
    out = str(tmp_path / "acc.pt")
    mp.spawn(_accum_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert torch.load(out, weights_only=True).tolist() == [True]


def _status_worker(rank, world, port, out_path):
    from factmx import functional as fxf
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = _ToyBlocks(seed=0)
        dp = DataParallel(net, bucket_mb=0.0002)
        st = fxf.device_status("cpu")
        got = []
        for fail in (True, False):
            st.zero_()
            dp.zero_grad()
            net(_videos()[rank]).pow(2).mean().backward()
            if fail and rank == 1:
                st[0] = 1                    # this rank's BiGRU backward timed out (FX_STATUS_GRU_TIMEOUT)
            dp.finish_gradients()
            got.append(int(st[0]))
        torch.save(torch.tensor(got), out_path + f".{rank}")
    finally:
        dist.destroy_process_group()


def test_data_parallel_spreads_a_failed_backward_to_every_rank(tmp_path):
    """A rank whose kernels set the device status word in the backward (invalid gradients, already in
    the all-reduced buckets) makes every rank see it after finish_gradients (MAX all-reduce of the word):
    every rank's FusedAdam then skips the update on the device and raises at its next read-back."""
    out = str(tmp_path / "st.pt")
    mp.spawn(_status_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        assert torch.load(out + f".{r}", weights_only=True).tolist() == [1, 0]


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N must start N ranks or refuse: never time one rank for an N-GPU request."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""          # no GPU visible (as in this container)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "refusing" in r.stderr, r.stderr[-2000:]
    env["WORLD_SIZE"] = "1"                  # a launcher that started fewer ranks than --gpus asks for
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]


class _NamesDataset:
    def __init__(self, n):
        self.names = [f"v{i}" for i in range(n)]

    def get_vnames(self):
        return self.names

    def __len__(self):
        return len(self.names)

    def __getitem__(self, v):
        i = int(v[1:])
        return torch.full((3, 2), float(i)).numpy(), [i] * 3, [i] * 3


def test_rank_sharded_loader_partitions_the_global_batch():
    from factmx.utils.dataset import DataLoader
    ds = _NamesDataset(10)
    loaders = [DataLoader(ds, 4, shuffle=True, rank=r, world_size=2, seed=7) for r in range(2)]
    ref = DataLoader(ds, 4, shuffle=True, rank=0, world_size=2, seed=7)
    for _ in range(2):                       # two epochs (reshuffle in between)
        for _ in range(len(ref)):
            parts = [next(ld) for ld in loaders]
            glob = ref.global_batch()
            assert parts[0][0] == glob[0::2] and parts[1][0] == glob[1::2]
            assert sorted(parts[0][0] + parts[1][0]) == sorted(glob)
        for ld in loaders:
            with pytest.raises(StopIteration):
                next(ld)
        with pytest.raises(StopIteration):
            ref.global_batch()
    with pytest.raises(ValueError):
        DataLoader(ds, 3, rank=0, world_size=2)
