"""The BiGRU recurrence kernels' scheduling variants produce the same numbers (GPU).

The forward's gate threads may sit on wave 0 writing their own tables (FX_GRU_STORE_WAVE=0), stage their
results for a fifth wave (1), or run on that fifth wave (2, the default); the granule gather may keep one
or two polls in flight per lane (FX_GRU_POLL2).  None of this changes an operation or its order, so the
outputs and every gradient must agree BITWISE across the variants (and with the fp64 reference of the
GRU within fp32 tolerance, which tests/test_gpu_kernels.py and test_gpu_long.py cover).  Library knobs
are read once per process: each variant runs in a child process that writes its tensors to a file."""
import os
import subprocess
import sys

import pytest
import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_ROOT, os.path.join(_ROOT, "fact-clip_amd")):     # (the child process has no conftest)
    if _p not in sys.path:
        sys.path.insert(0, _p)

pytestmark = pytest.mark.gpu

VARIANTS = [{"FX_GRU_STORE_WAVE": "2", "FX_GRU_POLL2": "1"},
            {"FX_GRU_STORE_WAVE": "1", "FX_GRU_POLL2": "1"},
            {"FX_GRU_STORE_WAVE": "0", "FX_GRU_POLL2": "0"}]


def _run(path):
    """Child: a ragged 3-sequence BiGRU (H = 512 -> 2 x 256) forward + backward; saves y and the grads."""
    from factmx import functional as fxf
    torch.manual_seed(0)
    gru = torch.nn.GRU(512, 256, 1, bidirectional=True).cuda()
    lens = [700, 1, 333]
    off = [0]
    for n in lens:
        off.append(off[-1] + n)
    x = torch.randn(off[-1], 512, device="cuda", requires_grad=True)
    g = torch.randn(off[-1], 512, device="cuda")
    y = fxf.gru(gru, x, seq_off=off)
    (y * g).sum().backward()
    out = {"y": y.detach().cpu(), "dx": x.grad.detach().cpu()}
    for n, p in gru.named_parameters():
        out[n] = p.grad.detach().cpu()
    torch.save(out, path)


def test_gru_scheduling_variants_bitwise(tmp_path):
    results = []
    for i, v in enumerate(VARIANTS):
        path = str(tmp_path / f"gru_{i}.pt")
        env = dict(os.environ, **v)
        p = subprocess.run([sys.executable, "-u", os.path.abspath(__file__), path], env=env, cwd=_ROOT, timeout=240)
        assert p.returncode == 0, (v, p.returncode)
        results.append(torch.load(path, weights_only=True))
    base = results[0]
    for v, r in zip(VARIANTS[1:], results[1:]):
        for k in base:
            assert torch.equal(base[k], r[k]), (v, k, (base[k] - r[k]).abs().max().item())


if __name__ == "__main__":
    _run(sys.argv[1])
