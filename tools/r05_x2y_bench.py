"""Round 5: X2Y_map forward + backward at the headline shapes (2 videos x 4096 frames, 32 action tokens,
hid 512, head 512), both directions, for a kernel trace of the backward pieces.

python tools/r05_x2y_bench.py [a2f|f2a] [iters]"""
import math
import os
import sys
import time

import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "fact-clip_amd")]
from factmx import functional as fxf  # noqa: E402

direction = sys.argv[1] if len(sys.argv) > 1 else "a2f"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
T, Q, nv, D, H, OUT = 4096, 32, 2, 512, 512, 512
g = torch.Generator().manual_seed(0)
tok = torch.randn(nv * Q, D, generator=g).cuda()
frm = torch.randn(nv * T, D, generator=g).cuda()
tpos, fpos = 0.5 * torch.randn_like(tok), 0.5 * torch.randn_like(frm)
if direction == "a2f":
    X, Y, Xp, Yp, xl, yl = tok, frm, tpos, fpos, [0, Q, 2 * Q], [0, T, 2 * T]
else:
    X, Y, Xp, Yp, xl, yl = frm, tok, fpos, tpos, [0, T, 2 * T], [0, Q, 2 * Q]
X, Y = X.requires_grad_(True), Y.requires_grad_(True)
W = {}
for n, shp in (("wk", (H, D)), ("bk", (H,)), ("wv", (H, D)), ("bv", (H,)), ("wq", (H, D)), ("bq", (H,)),
               ("wy", (OUT, D + H)), ("by", (OUT,))):
    W[n] = (torch.randn(*shp, generator=g) / math.sqrt(shp[-1])).cuda().requires_grad_(True)
gout = torch.randn(nv * (T if direction == "a2f" else Q), OUT).cuda()
for it in range(iters):
    out, logit, attn = fxf.X2YFn.apply(X, Y, Xp, Yp, (xl, yl), W["wk"], W["bk"], W["wv"], W["bv"], W["wq"], W["bq"],
                                       W["wy"], W["by"], 0.0, 0)
    ((out * gout).sum() + logit.sum() * 1e-3).backward()
    if it == 2:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
torch.cuda.synchronize()
print(direction, f"{1e3 * (time.perf_counter() - t0) / (iters - 3):.3f} ms per fwd+bwd")
