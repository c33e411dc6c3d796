"""Round 5: the cross-attention projection GEMMs alone, at the headline step's shapes, for rocprofv3 PMC
passes (FETCH_SIZE / WRITE_SIZE per dispatch: every dispatch of this script is the named GEMM).

python tools/r05_xattn_pmc.py kv|x2y   -- SCA frame-memory K/V projection (8192 x 512 -> 3072) or one X2Y
frame-side projection (8192 x 512 -> 512); 20 launches through factmx.functional.linear."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "fact-clip_amd")]
from factmx import functional as fxf  # noqa: E402

T, Hm = 8192, 512
N = {"kv": 3072, "x2y": 512}[sys.argv[1]]
g = torch.Generator().manual_seed(0)
x = torch.randn(T, Hm, generator=g).cuda()
w = (torch.randn(N, Hm, generator=g) * Hm ** -0.5).cuda()
b = torch.zeros(N).cuda()
with torch.no_grad():
    for _ in range(20):
        y = fxf.linear(x, w, b)
torch.cuda.synchronize()
print(sys.argv[1], tuple(y.shape), float(y.abs().mean()))
