"""Diagnostic: device time of each op group of the benchmark step, in isolation (fwd and bwd).

python tools/op_bench.py [--iters 20]
Builds the bench model (bench.make_cfg / build_model, 2 videos x T=4096) and times, with HIP events
on the current stream, the decoders, the X2Y layers, the MS-TCN stacks and the GRU of each block on
inputs of the bench shapes.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from factmx import functional as fxf  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def fwd_bwd(make, iters):
    """(fwd us, bwd us) of out = make(); out.backward(g)."""
    def f():
        with torch.no_grad():
            make()
    fwd = timed(f, iters)
    state = {}

    def setup():
        out = make()
        state["out"], state["g"] = out, torch.ones_like(out)

    def b():
        state["out"].backward(state["g"], retain_graph=True)
    setup()
    bwd = timed(b, iters)
    return fwd, bwd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    cfg = bench.make_cfg()
    T, D, C, nv = 4096, 2048, 75, 2
    net, _ = bench.build_model(cfg, D, C, device="cuda", seed=0)
    net.train()
    dev = "cuda"
    Q = cfg.FACT.ntoken
    rows = []
    b0 = net.block_list[0]
    H = cfg.Bi.hid_dim
    A = cfg.Bi.a_dim
    feats = torch.randn(nv * T, D, device=dev, requires_grad=True)
    frames = torch.randn(nv * T, H, device=dev, requires_grad=True)
    toks = torch.randn(nv * Q, A, device=dev, requires_grad=True)
    apos = net.action_query.squeeze(1).repeat(nv, 1).detach()
    rows.append(("block0 MS-TCN (in_map 2048->256, 10 layers)",
                 fwd_bwd(lambda: fxf.mstcn(b0.frame_branch, feats, T=T, nvid=nv), args.iters)))
    rows.append(("block0 SCA decoder (6 layers, CA over T)",
                 fwd_bwd(lambda: fxf.decoder(b0.action_branch, toks, frames, pos=None, query_pos=apos, nvid=nv),
                         args.iters)))
    b1 = net.block_list[1]
    vb_rows = ([v * T for v in range(nv + 1)], [v * Q for v in range(nv + 1)])
    rows.append(("block1 f2a X2Y (frames -> tokens)",
                 fwd_bwd(lambda: fxf.x2y(b1.f2a_layer, frames, toks, None, apos, rows=vb_rows)[0], args.iters)))
    rows.append(("block1 SA decoder (1 layer)",
                 fwd_bwd(lambda: fxf.decoder(b1.action_branch, toks, None, query_pos=apos, nvid=nv), args.iters)))
    tok_out = torch.randn(nv * Q, A + C + 1, device=dev, requires_grad=True)
    rows.append(("block1 a2f X2Y (tokens -> frames)",
                 fwd_bwd(lambda: fxf.x2y(b1.a2f_layer, tok_out, frames, apos, None,
                                         rows=(vb_rows[1], vb_rows[0]))[0], args.iters)))
    fin = torch.randn(nv * T, cfg.Bu.f_dim if cfg.Bu.f_dim else H, device=dev, requires_grad=True)
    rows.append(("block1 MS-TCN (10 layers)",
                 fwd_bwd(lambda: fxf.mstcn(b1.frame_branch, fin, T=T, nvid=nv), args.iters)))
    b2 = net.block_list[2]
    S = [103, 27]
    seg = torch.randn(sum(S), H, device=dev, requires_grad=True)
    rows.append(("block2 GRU (S = 103 + 27)",
                 fwd_bwd(lambda: fxf.gru(b2.seg_update, seg, seq_off=[0, S[0], S[0] + S[1]]), args.iters)))
    tot_f = tot_b = 0.0
    for name, (f, b) in rows:
        print(f"{name:48s} fwd {f:9.1f} us   bwd {b:9.1f} us")
        tot_f += f
        tot_b += b
    print(f"{'(sum)':48s} fwd {tot_f:9.1f} us   bwd {tot_b:9.1f} us")


if __name__ == "__main__":
    main()
