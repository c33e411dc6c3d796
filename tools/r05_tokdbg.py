"""Round-5 debug: the SCA decoder forward through the token kernel vs the separate launches
(run twice: FX_DEC_TOK=1 / 0), outputs + saved buffer written to gpurun_out/tokdbg_<tok>.pt."""
import os
import sys

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "fact-clip_amd")]
from factmx.models import basic  # noqa: E402
from factmx import functional as fxf  # noqa: E402

DEV = "cuda"
R, A, h, FF, Hm, L, T = int(os.environ.get("R", "32")), 256, 8, 512, 512, int(os.environ.get("NL", "6")), 1024
layer = basic.SCALayer(A, Hm, h, FF, dropout=0.0, attn_dropout=0.0)
dec = basic.SCADecoder(A, A, 2 * A, layer, L, norm=torch.nn.LayerNorm(A), in_map=False)
g = torch.Generator().manual_seed(1)
with torch.no_grad():
    for n, p in dec.named_parameters():
        p.copy_(torch.randn(p.shape, generator=g) * (0.5 if "norm" in n else p.shape[-1] ** -0.5) +
                (1.0 if "norm" in n and n.endswith("weight") else 0.0))
dec = dec.to(DEV).train()
tgt = torch.randn(R, 1, A, generator=g).to(DEV).requires_grad_(True)
mem = torch.randn(T, 1, Hm, generator=g).to(DEV).requires_grad_(True)
qpos = torch.randn(R, 1, A, generator=g).to(DEV).requires_grad_(True)
out = dec(tgt, mem, pos=None, query_pos=qpos)
node = out.grad_fn
while node is not None and "DecoderFn" not in type(node).__name__:
    node = node.next_functions[0][0]
saved = node.saved_tensors[4]
torch.cuda.synchronize()
st = fxf.device_status(tgt.device)
print("tok", os.environ.get("FX_DEC_TOK", "1"), "out absmax", out.abs().max().item(), "status", st.tolist())
out.sum().backward()
torch.cuda.synchronize()
print("grads tgt", tgt.grad.abs().max().item(), "mem", mem.grad.abs().max().item(), "status", st.tolist())
torch.save({"out": out.detach().cpu(), "saved": None if saved is None else saved.detach().cpu(),
            "gt": tgt.grad.cpu(), "gm": mem.grad.cpu(),
            "gp": {n: p.grad.cpu() for n, p in dec.named_parameters()}},
           f"gpurun_out/tokdbg_{os.environ.get('FX_DEC_TOK', '1')}.pt")
