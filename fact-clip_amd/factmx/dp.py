"""Data parallelism over whole videos (one process per GPU, RCCL over xGMI).

The reference has no distributed code; its batch is a
loop over B=1 videos whose losses are averaged (blocks.py:913-915).  Sharding
the videos over ranks and averaging gradients is therefore exactly equivalent
for equal per-rank counts.

``DataParallel`` makes every parameter's ``.grad`` a view into ONE flat fp32
buffer (the HIP kernels accumulate weight gradients straight into those views),
laid out in parameter order, so the parameters of each FACT block are one
contiguous slice.  Those slices are the all-reduce buckets: the model marks the
input of every block during the forward (``mark_block_input``); when autograd
has produced the gradient of block k's input, every kernel of block k's backward
has been enqueued, so its bucket's all-reduce is launched right there
(asynchronously, from a collective stream that waits on events recorded on the
compute stream and on the library's side stream -- where block k's deferred
weight-gradient GEMMs run -- so neither of those streams ever waits for the
other mid-backward) and runs over xGMI while blocks k-1 .. 0 compute their
backward.  ``finish_gradients``
launches what is left (block 0, the action queries and the CLIP projection head,
whose gradients are only final at the end) and makes the compute stream wait
for all of them -- no host synchronisation.  Buckets are few and large (xGMI
rings are per-link bandwidth bound).  Rank 0's weights are broadcast once at
construction, so every rank starts from identical parameters whatever its seed.

``FlatGradReducer`` is the same flat buffer without per-block buckets (one or
more equal buckets reduced after backward), for models without a block list.
"""
import time

import torch
import torch.distributed as dist

from . import functional as fxf


def _dist_world(group=None):
    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


def _flat_grads(params):
    dev = params[0].device
    total = sum(p.numel() for p in params)
    flat = torch.zeros(total, device=dev, dtype=params[0].dtype)
    off = 0
    for p in params:
        n = p.numel()
        p.grad = flat[off:off + n].view_as(p)
        off += n
    return flat


def _check_views(params, flat):
    lo = flat.data_ptr()
    hi = lo + flat.numel() * flat.element_size()
    for p in params:
        if p.grad is None or not (lo <= p.grad.data_ptr() < hi):
            raise RuntimeError("parameter .grad was detached from the flat buffer (use zero_grad here, "
                               "not optimizer.zero_grad(set_to_none=True))")


def _all_reduce_mean_async(t, group):
    """Launch an all-reduce (mean) of t; returns (work, needs_div)."""
    if dist.get_backend(group) == "nccl":      # RCCL averages inside the collective
        return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group, async_op=True), False
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=True), True


class FlatGradReducer:
    def __init__(self, params, bucket_mb=64, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.flat = _flat_grads(self.params)
        total = self.flat.numel()
        per = max(1, int(bucket_mb * (1 << 20) // self.flat.element_size()))
        self.buckets = [self.flat[i:i + per] for i in range(0, total, per)]

    def zero_grad(self):
        """Zero in place (keeps the .grad views; never set grads to None).  The views are
        re-verified every 64th call only (a Python loop over 400+ tensors is host time)."""
        self.flat.zero_()
        self._calls = getattr(self, "_calls", -1) + 1
        if self._calls % 64 == 0:
            _check_views(self.params, self.flat)

    def all_reduce_mean(self):
        world = _dist_world(self.group)
        if world == 1:
            return
        works = [_all_reduce_mean_async(b, self.group) for b in self.buckets]
        for w, _ in works:
            w.wait()
        if works and works[0][1]:
            self.flat.div_(world)


def _merge_adjacent(buckets):
    """Views of one flat buffer, merged where one ends exactly where the next begins."""
    out = []
    for b in sorted(buckets, key=lambda t: t.data_ptr()):
        if out and out[-1].data_ptr() + out[-1].numel() * out[-1].element_size() == b.data_ptr():
            p = out[-1]
            base = p._base if p._base is not None else p
            off = (p.data_ptr() - base.data_ptr()) // p.element_size()
            out[-1] = base.view(-1)[off:off + p.numel() + b.numel()]
        else:
            out.append(b)
    return out


def mark_block_input(net, k, x):
    """Called by the model's forward with the input tensor of block k: registers the hook that
    launches block k's gradient bucket once autograd has produced x's gradient."""
    dp = getattr(net, "_fx_dp", None)
    if dp is None or not dp.active or not torch.is_grad_enabled() or not torch.is_tensor(x) or not x.requires_grad:
        return
    dp._arm(k, x)


def mark_block_part(net, k, name, x):
    """Called by block k's forward with a tensor x that only sub-module `name` of the block (and what
    follows it) consumes -- e.g. the input block's frame-branch output, read by its action branch: once
    autograd has produced x's gradient, every kernel of `name`'s backward has been enqueued, so that
    part of block k's bucket launches right there instead of with the rest of the block.  Needed where
    the block's own input has no gradient (the first block reads the data), so its bucket would
    otherwise wait for the end of the backward."""
    dp = getattr(net, "_fx_dp", None)
    if dp is None or not dp.active or not torch.is_grad_enabled() or not torch.is_tensor(x) or not x.requires_grad:
        return
    dp._arm_part(k, name, x)


class DataParallel:
    """Whole-video data parallelism for FACT / FACT_CLIP (or any module with a ``block_list``).

    dp = DataParallel(net)                 # broadcast rank 0's weights, flat grad buckets
    dp.zero_grad(); loss = net(...)[0]; loss.backward(); dp.finish_gradients()
    optimizer over dp.flat (factmx.optim.FusedAdam(..., grad_flat=dp.flat))
    """

    def __init__(self, net, group=None, broadcast=True, bucket_mb=256, force_buckets=False):
        self.net = net
        self.group = group
        self.world = _dist_world(group)
        # force_buckets: keep the per-block bucket schedule (hooks, collective stream, all-reduces)
        # even in a one-rank group -- how the RCCL path is exercised and its overhead measured on a
        # single GPU (tests/test_gpu_rccl.py, bench.py dp_schedule_overhead_ms)
        if force_buckets and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("DataParallel(force_buckets=True) needs an initialised process group")
        self.active = self.world > 1 or bool(force_buckets)
        named = [(n, p) for n, p in net.named_parameters() if p.requires_grad]
        self.params = [p for _, p in named]
        if broadcast and self.world > 1:
            self._broadcast_from_rank0()
        self.flat = _flat_grads(self.params)
        # contiguous parameter range of every block (parameter order = registration order)
        nblk = len(getattr(net, "block_list", []))
        ranges = {}
        off = 0
        for n, p in named:
            parts = n.split(".")
            if parts[0] == "block_list" and len(parts) > 1 and parts[1].isdigit():
                k = int(parts[1])
                lo, hi = ranges.get(k, (off, off))
                if hi != off:
                    raise RuntimeError(f"block {k} parameters are not contiguous in parameter order")
                ranges[k] = (lo, off + p.numel())
            off += p.numel()
        per = max(1, int(bucket_mb * (1 << 20) // 4))

        def cut(lo, hi):
            return [self.flat[i:min(i + per, hi)] for i in range(lo, hi, per)]

        def span(prefix):
            """[lo, hi) of the parameters named prefix.* (contiguous in parameter order), or None."""
            lo = hi = None
            off = 0
            for n, p in named:
                if n.startswith(prefix + "."):
                    if lo is None:
                        lo = off
                    elif hi != off:
                        raise RuntimeError(f"{prefix} parameters are not contiguous in parameter order")
                    hi = off + p.numel()
                off += p.numel()
            return None if lo is None else (lo, hi)

        # parts of a block launched by their own hook (mark_block_part): the sub-modules the block lists
        # in dp_parts; the block's bucket keeps the rest of its range
        blocks = list(getattr(net, "block_list", []))
        self.part_buckets = {}
        self.block_buckets = {}
        for k, (lo, hi) in ranges.items():
            cuts = []
            for name in getattr(blocks[k], "dp_parts", ()) if k < len(blocks) else ():
                sp = span(f"block_list.{k}.{name}")
                if sp is not None:
                    self.part_buckets[(k, name)] = cut(*sp)
                    cuts.append(sp)
            rem, cur = [], lo
            for a, b in sorted(cuts) + [(hi, hi)]:
                rem += cut(cur, a)
                cur = b
            self.block_buckets[k] = rem
        # everything outside the blocks (action queries, CLIP projection head): the tail buckets, except
        # the modules the model lists in dp_head_modules -- used only after the last block, so their
        # gradients are final once the backward is under way: they go with the first hook that fires
        heads = [sp for sp in (span(n) for n in getattr(net, "dp_head_modules", ())) if sp is not None]
        rest, cur = [], 0
        for lo, hi in sorted(list(ranges.values()) + heads) + [(self.flat.numel(), self.flat.numel())]:
            rest += cut(cur, lo)
            cur = hi
        self.rest_buckets = rest
        self.head_buckets = [b for sp in heads for b in cut(*sp)]
        self.tail_bytes = 0          # bytes finish_gradients reduced (after the backward), last step
        self.nblk = nblk
        self._pending = []
        self._launched = set()
        self.hook_launched = []
        self._armed = {}
        self._calls = -1
        self.host_issue_s = 0.0      # host time spent issuing bucket collectives (diagnostics)
        self.issue_thread = False    # make the collective calls from a helper thread (A/B knob)
        self._q = None
        self._worker_error = None
        # the stream the bucket collectives are issued from: it waits for the compute stream (block k's
        # input-gradient chain) and the library's side stream (block k's deferred weight gradients) at
        # the bucket's launch, so the compute stream itself never waits mid-backward
        dev = self.flat.device
        self._cstream = torch.cuda.Stream(device=dev) if (self.active and dev.type == "cuda") else None
        if self.active:
            net._fx_dp = self
        elif getattr(net, "_fx_dp", None) is not None:
            net._fx_dp = None

    @torch.no_grad()
    def _broadcast_from_rank0(self):
        flat = torch.cat([p.detach().reshape(-1) for p in self.params])
        dist.broadcast(flat, 0, group=self.group)
        off = 0
        for p in self.params:
            p.copy_(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        for b in self.net.buffers():
            if b.is_floating_point():
                dist.broadcast(b, 0, group=self.group)

    def zero_grad(self):
        self.flat.zero_()
        self._pending = []
        self._launched = set()
        self.hook_launched = []
        self._armed = {}
        self._heads_out = False
        self._calls += 1
        if self._calls % 64 == 0:
            _check_views(self.params, self.flat)

    def _arm(self, k, x):
        # one arm per video that ran block k (the per-video path runs the blocks once per video):
        # the bucket launches when the LAST of them has its input gradient
        if k in self._launched:
            # a second backward without zero_grad would add unreduced gradients on top of reduced ones
            raise RuntimeError("factmx DataParallel: each step must be zero_grad(), one forward + backward, "
                               "finish_gradients(); gradient accumulation over several backward passes "
                               "between zero_grad() calls is not supported")
        if k in self.block_buckets:
            self._armed[k] = self._armed.get(k, 0) + 1
            x.register_hook(lambda g, k=k: self._fired(k))

    def _arm_part(self, k, name, x):
        key = (k, name)
        if key in self._launched:
            raise RuntimeError("factmx DataParallel: each step must be zero_grad(), one forward + backward, "
                               "finish_gradients()")
        if key in self.part_buckets:
            self._armed[key] = self._armed.get(key, 0) + 1
            x.register_hook(lambda g, key=key: self._fired(key))

    def _fired(self, k):
        self._armed[k] -= 1
        if self._armed[k] == 0:
            self._launch_heads()
            self._launch_block(k, True)

    def _launch_heads(self):
        if not getattr(self, "_heads_out", False):
            self._heads_out = True
            self._issue(self.head_buckets)

    def _issue(self, buckets):
        """All-reduce `buckets` from the collective stream once everything enqueued so far on the
        compute stream AND on the library's side stream has run (the side stream carries weight
        gradients deferred past their block's backward call).  Only the collective stream waits; the
        collective itself (RCCL's own stream) is ordered after it by torch.distributed.  With
        ``issue_thread`` the hook only records the two events and a helper thread makes the
        collective calls, so the autograd thread goes straight back to enqueueing the backward."""
        if not buckets:
            return
        t0 = time.perf_counter()
        try:
            cs = self._cstream
            if cs is None:                   # CPU tensors (gloo tests): nothing to order
                for b in buckets:
                    self._pending.append(_all_reduce_mean_async(b, self.group))
                return
            evs = [torch.cuda.current_stream(cs.device).record_event()]
            side = fxf.side_stream()
            if side is not None:
                evs.append(side.record_event())
            if self.issue_thread:
                self._worker().put((buckets, evs))
            else:
                self._issue_after(buckets, evs)
        finally:
            self.host_issue_s += time.perf_counter() - t0

    def _issue_after(self, buckets, evs):
        cs = self._cstream
        for e in evs:
            cs.wait_event(e)
        with torch.cuda.stream(cs):
            for b in buckets:
                self._pending.append(_all_reduce_mean_async(b, self.group))

    def _worker(self):
        if self._q is None:
            import queue
            import threading
            self._q = queue.Queue()
            dev = self._cstream.device

            def run():
                torch.cuda.set_device(dev)
                while True:
                    item = self._q.get()
                    try:
                        if item is None:
                            return
                        self._issue_after(*item)
                    except BaseException as e:      # re-raised on the caller's thread at finish
                        self._worker_error = e
                    finally:
                        self._q.task_done()
            self._thread = threading.Thread(target=run, name="factmx-dp-issue", daemon=True)
            self._thread.start()
        return self._q

    def _issue_status(self):
        """All-reduce (MAX) the device status word behind the gradient buckets, on the device: a rank
        whose BiGRU timed out in this backward (invalid gradients, already summed into the buckets) makes
        EVERY rank's FusedAdam skip the update (fx_adam_step_checked reads the word) and every rank raise
        at its next read-back, so the replicas neither apply corrupted averages nor diverge."""
        if self.world <= 1:
            return
        st = fxf.device_status(self.flat.device)[:1]
        cs = self._cstream
        if cs is None:
            self._pending.append((dist.all_reduce(st, op=dist.ReduceOp.MAX, group=self.group, async_op=True), False))
            return
        cs.wait_stream(torch.cuda.current_stream(cs.device))
        with torch.cuda.stream(cs):
            self._pending.append((dist.all_reduce(st, op=dist.ReduceOp.MAX, group=self.group, async_op=True), False))

    def _launch_block(self, k, from_hook=False):
        """k: a block index (its bucket less its parts) or a (block, part) key."""
        if not self.active or k in self._launched:
            return
        self._launched.add(k)
        if from_hook:
            self.hook_launched.append(k)
        self._issue(self.part_buckets.get(k, []) if isinstance(k, tuple) else self.block_buckets.get(k, []))

    def finish_gradients(self):
        """Launch the buckets no hook has launched and make the current stream wait for all of them."""
        if not self.active:
            return
        # the buckets no hook launched (block 0: its input is the data) and the tail (action queries,
        # CLIP head): adjacent slices of the flat buffer are merged into one collective
        left = [b for k in sorted(self.block_buckets, reverse=True) if k not in self._launched
                for b in self.block_buckets[k]]
        left += [b for key in sorted(self.part_buckets, reverse=True) if key not in self._launched
                 for b in self.part_buckets[key]]
        if not getattr(self, "_heads_out", False):
            left += self.head_buckets
            self._heads_out = True
        self._launched.update(self.block_buckets)
        self._launched.update(self.part_buckets)
        fxf.side_join()           # (the backward's end-of-pass callback has normally joined already)
        tail = _merge_adjacent(left + list(self.rest_buckets))
        self.tail_bytes = sum(b.numel() * b.element_size() for b in tail)
        self._issue(tail)
        self._issue_status()
        if self._q is not None:
            self._q.join()        # every collective has been issued (the helper thread is idle)
            if self._worker_error is not None:
                e, self._worker_error = self._worker_error, None
                raise e
        need_div = False
        for w, div in self._pending:
            w.wait()
            need_div = need_div or div
        self._pending = []
        if need_div:
            self.flat.div_(self.world)
