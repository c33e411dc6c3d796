"""The fused MS-TCN layer kernel's scheduling variants produce the same numbers (GPU).

Stage pairs per barrier with A fragments read one pair ahead (FX_FRL_PAIR=1, the default) or one barrier
per 32-deep stage (0), and the row tiles in XCD runs that follow the conv taps (FX_FRL_XCD=2, default),
plain XCD runs (1) or dispatch order (0): none of them changes an operation or the k order of any
accumulation, so the MS-TCN output, its input gradient and every weight gradient agree BITWISE across the
variants (the fp64 comparison itself is tests/test_gpu_kernels.py::test_mstcn_fused_layers_match_fp64).
Library knobs are read once per process: each variant runs in a child process."""
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

VARIANTS = [{"FX_FRL_PAIR": "1", "FX_FRL_XCD": "2"},
            {"FX_FRL_PAIR": "0", "FX_FRL_XCD": "2"},
            {"FX_FRL_PAIR": "1", "FX_FRL_XCD": "0"},
            {"FX_FRL_PAIR": "1", "FX_FRL_XCD": "1"}]


def _run(path):
    """Child: a 10-layer F = 256 MS-TCN over 2 x 4096 rows (the fused layer in both directions)."""
    from factmx import functional as fxf
    from factmx.dp import FlatGradReducer
    from factmx.models.basic import MSTCN
    fxf.MSTCN_FUSED_LAYERS = 2
    torch.manual_seed(0)
    mod = MSTCN(64, 256, 40, 10, dropout=0.0, ln=False, in_map=True).cuda().train()
    FlatGradReducer(mod.parameters())
    x = torch.randn(8192, 64, device="cuda", requires_grad=True)
    g = torch.randn(8192, 40, device="cuda")
    y = fxf.mstcn(mod, x, T=4096, nvid=2)
    (y * g).sum().backward()
    out = {"y": y.detach().cpu(), "dx": x.grad.detach().cpu()}
    for n, p in mod.named_parameters():
        out[n] = p.grad.detach().cpu()
    torch.save(out, path)


def test_fused_layer_scheduling_variants_bitwise(tmp_path):
    results = []
    for i, v in enumerate(VARIANTS):
        path = str(tmp_path / f"frl_{i}.pt")
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
