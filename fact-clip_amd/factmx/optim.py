"""Flat-buffer train-step tail: clip_grad_norm_ + Adam in two HIP launches (scripts/train.py:265-267).

The reference step is ``clip_grad_norm_(net.parameters(), cfg.clip_grad_norm)`` then
``torch.optim.Adam.step()`` (train_tools/train.py via scripts/train.py:262-268).  With 400+
parameter tensors that is ~20 multi-tensor launches plus per-tensor host work per step.
``FusedAdam`` keeps parameters, gradients and both moment buffers as single flat fp32 buffers
(parameters are re-pointed into the flat storage once, ``param.grad`` are views into the
gradient buffer shared with ``factmx.dp.FlatGradReducer``) and runs the whole tail as
``fx_adam_step``: deterministic g^2 partial sums, then one fused clip + Adam update.  Semantics
are torch.optim.Adam's (amsgrad off, L2 weight decay) and clip_grad_norm_'s (2-norm,
coefficient min(max_norm / (norm + 1e-6), 1), clipped gradient left in ``.grad``).
"""
import torch

from . import native as nx


def flatten_parameters(params):
    """Re-point every parameter's storage into one contiguous fp32 buffer (same values, same
    Parameter objects, so modules, state_dict and the kernels see no difference)."""
    params = [p for p in params if p.requires_grad]
    dev = params[0].device
    total = sum(p.numel() for p in params)
    flat = torch.empty(total, device=dev, dtype=torch.float32)
    off = 0
    with torch.no_grad():
        for p in params:
            n = p.numel()
            flat[off:off + n].copy_(p.reshape(-1))
            p.data = flat[off:off + n].view_as(p)
            off += n
    return flat, params


class FusedAdam:
    """torch.optim.Adam(params, lr, betas, eps, weight_decay) with an optional fused
    clip_grad_norm_(max_grad_norm), over flat buffers.  ``grad_flat`` is the flat gradient
    buffer whose views are the parameters' ``.grad`` in the same order (FlatGradReducer.flat);
    without it one is created here."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, max_grad_norm=None,
                 grad_flat=None):
        self.flat, self.params = flatten_parameters(params)
        n = self.flat.numel()
        if grad_flat is None:
            grad_flat = torch.zeros(n, device=self.flat.device)
            off = 0
            for p in self.params:
                p.grad = grad_flat[off:off + p.numel()].view_as(p)
                off += p.numel()
        assert grad_flat.numel() == n and grad_flat.is_contiguous()
        off = 0
        for p in self.params:
            g = p.grad
            if g is None or g.data_ptr() != grad_flat.data_ptr() + 4 * off:
                raise ValueError("FusedAdam: parameter .grad must be views into grad_flat in parameter order")
            off += p.numel()
        self.grad_flat = grad_flat
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.exp_avg = torch.zeros_like(self.flat)
        self.exp_avg_sq = torch.zeros_like(self.flat)
        self.step_count = 0
        lib = nx.load()
        self._ws = torch.empty(lib.fx_grad_norm_workspace_floats(), device=self.flat.device)
        self.total_norm = torch.zeros(1, device=self.flat.device)

    @torch.no_grad()
    def step(self):
        lib = nx.load()
        self.step_count += 1
        mx = float(self.max_grad_norm) if self.max_grad_norm else 0.0
        b1, b2 = self.betas
        # guarded by the device status word: a step whose kernels failed (BiGRU timeout in the backward)
        # leaves the parameters and moments untouched; the failure is raised by the next status read-back
        from .functional import device_status
        nx.check(lib.fx_adam_step_checked(nx.ptr(self.flat), nx.ptr(self.grad_flat), nx.ptr(self.exp_avg),
                                          nx.ptr(self.exp_avg_sq), self.flat.numel(), self.step_count,
                                          float(self.lr), float(b1), float(b2), float(self.eps),
                                          float(self.weight_decay), mx, nx.ptr(self._ws), nx.ptr(self.total_norm),
                                          nx.ptr(device_status(self.flat.device)), nx.stream()),
                 "fx_adam_step_checked")

    def zero_grad(self, set_to_none=False):
        self.grad_flat.zero_()

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg.clone(), "exp_avg_sq": self.exp_avg_sq.clone(),
                "lr": self.lr, "betas": self.betas, "eps": self.eps, "weight_decay": self.weight_decay,
                "max_grad_norm": self.max_grad_norm}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])


def clip_grad_norm_flat_(grad_flat, max_norm):
    """clip_grad_norm_ over one flat gradient buffer (two launches, no host sync); returns the
    total norm as a 1-element device tensor."""
    lib = nx.load()
    ws = torch.empty(lib.fx_grad_norm_workspace_floats(), device=grad_flat.device)
    norm = torch.empty(1, device=grad_flat.device)
    nx.check(lib.fx_grad_norm(nx.ptr(grad_flat), grad_flat.numel(), nx.ptr(ws), nx.ptr(norm), nx.stream()),
             "fx_grad_norm")
    nx.check(lib.fx_clip_grad_scale(nx.ptr(grad_flat), grad_flat.numel(), nx.ptr(ws), float(max_norm), nx.stream()),
             "fx_clip_grad_scale")
    return norm
