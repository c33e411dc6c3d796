"""Round-4 micro-benchmark: BiGRU (fxf.gru, gru.hip) time per recurrent step, forward and backward.

nn.GRU(512, 256, bidirectional) as UpdateBlockTDU.seg_update (blocks.py:401,432), `nseq` sequences of S
steps stacked by rows (the lockstep batch's videos).  Per-step cost = slope of the launch time over S
(HIP events around the autograd call; the input / weight GEMMs are S-proportional too but small).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
import torch  # noqa: E402


def main():
    from factmx import functional as fxf
    torch.manual_seed(0)
    gru = torch.nn.GRU(512, 256, 1, bidirectional=True).cuda()
    nseq = int(os.environ.get("NSEQ", 2))
    res = {}
    for S in (100, 400, 1600, 3400):
        x = torch.randn(nseq * S, 512, device="cuda", requires_grad=True)
        off = [S * i for i in range(nseq + 1)]
        fw, bw = [], []
        for it in range(6):
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            for p in gru.parameters():
                p.grad = None
            x.grad = None
            e0.record()
            y = fxf.gru(gru, x, seq_off=off if nseq > 1 else None)
            e1.record()
            y.backward(torch.ones_like(y))
            e2.record()
            torch.cuda.synchronize()
            if it >= 2:
                fw.append(e0.elapsed_time(e1))
                bw.append(e1.elapsed_time(e2))
        res[S] = (min(fw), min(bw))
        print(f"S={S:5d} nseq={nseq}: fwd {res[S][0] * 1e3:9.1f} us  bwd {res[S][1] * 1e3:9.1f} us", flush=True)
    s0, s1 = 100, 3400
    print(f"per recurrent step: fwd {(res[s1][0] - res[s0][0]) * 1e3 / (s1 - s0):.3f} us, "
          f"bwd {(res[s1][1] - res[s0][1]) * 1e3 / (s1 - s0):.3f} us", flush=True)


if __name__ == "__main__":
    main()
