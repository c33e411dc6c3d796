"""Round-5 debug: structured inputs through fx_tok_gemm (identity weights, one-hot rows) -> gpurun_out/tokgemm.pt"""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "fact-clip_amd")]
from factmx import functional as fxf  # noqa: E402
from factmx import native as nx  # noqa: E402

DEV = "cuda"
lib = nx.load()
out = {}
M, N, K = 64, 256, 256
a = (torch.arange(M, dtype=torch.float32)[:, None] * 1000 + torch.arange(K, dtype=torch.float32)[None, :]).to(DEV)
for name, w in (("eye", torch.eye(N, K)), ("rand", torch.randn(N, K) / 16)):
    w = w.float().to(DEV).contiguous()
    c = torch.zeros(M, N, device=DEV)
    st = fxf.device_status(c.device)
    rc = lib.fx_tok_gemm(nx.ptr(a), K, M, N, K, 0, None, None, nx.ptr(w), K, 0, None, None, 0, nx.ptr(c), N, nx.ptr(st),
                         nx.stream())
    torch.cuda.synchronize()
    out[name] = (a.cpu(), w.cpu(), c.cpu(), rc, st.tolist())
    print(name, rc, st.tolist(), (c - a @ w.t()).abs().max().item())
torch.save(out, "gpurun_out/tokgemm.pt")
