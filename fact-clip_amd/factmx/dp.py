"""Data parallelism over whole videos (one process per GPU, RCCL over xGMI).

The reference has no distributed code; its batch is a
loop over B=1 videos whose losses are averaged (blocks.py:913-915).  Sharding
the videos over ranks and averaging gradients is therefore exactly equivalent
for equal per-rank counts.

``FlatGradReducer`` makes every parameter's ``.grad`` a view into a few large
contiguous buckets, so backward accumulates straight into the communication
buffers and the exchange is a handful of large all-reduces (xGMI rings are
per-link bandwidth bound: few, big messages).  Buckets are launched
asynchronously as soon as backward finishes; clip-grad-norm then runs on the
identical reduced gradients on every rank with no extra collective.
"""
import torch
import torch.distributed as dist


class FlatGradReducer:
    def __init__(self, params, bucket_mb=64, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        dev = self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, device=dev, dtype=self.params[0].dtype)
        off = 0
        for p in self.params:
            n = p.numel()
            p.grad = self.flat[off:off + n].view_as(p)
            off += n
        per = max(1, int(bucket_mb * (1 << 20) // self.flat.element_size()))
        self.buckets = [self.flat[i:i + per] for i in range(0, total, per)]

    def zero_grad(self):
        """Zero in place (keeps the .grad views; never set grads to None).  The views are
        re-verified every 64th call only (a Python loop over 400+ tensors is host time)."""
        self.flat.zero_()
        self._calls = getattr(self, "_calls", -1) + 1
        if self._calls % 64:
            return
        for p in self.params:
            if p.grad is None or p.grad.data_ptr() < self.flat.data_ptr() or \
                    p.grad.data_ptr() >= self.flat.data_ptr() + self.flat.numel() * self.flat.element_size():
                raise RuntimeError("parameter .grad was detached from the flat buffer (use zero_grad here, "
                                   "not optimizer.zero_grad(set_to_none=True))")

    def all_reduce_mean(self):
        if not (dist.is_available() and dist.is_initialized()):
            return
        world = dist.get_world_size(self.group)
        if world == 1:
            return
        if dist.get_backend(self.group) == "nccl":
            # RCCL averages in the collective itself (no extra scale launch)
            works = [dist.all_reduce(b, op=dist.ReduceOp.AVG, group=self.group, async_op=True) for b in self.buckets]
            for w in works:
                w.wait()
            return
        works = [dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group, async_op=True) for b in self.buckets]
        for w in works:
            w.wait()
        self.flat.div_(world)
