"""Diagnostic: where one fused MS-TCN layer launch (frl_kernel) spends its time, from s_memrealtime stamps of
thread 0 of every workgroup (diagnostic build: mstcn_fused.hip with -DFRL_STAMPS, loaded through FACTMX_LIB).
Runs a 10-layer F=256 MS-TCN forward on 2 x 4096 rows and prints, for the last layer's launch, the spread of
each interval over the 256 workgroups (us):
  0 start -> 1 prologue loads issued -> 2 first barrier -> 3 phase-1 loop done -> 4 phase-1 epilogue (V tile,
  residual loads) -> 5 barrier -> 6 phase-2 loop done -> 7 phase-2 epilogue stores issued."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from factmx import functional as fxf  # noqa: E402
from factmx import native as nx  # noqa: E402
from factmx.models.basic import MSTCN  # noqa: E402


def main():
    torch.manual_seed(0)
    mod = MSTCN(256, 256, 256, 10, dropout=0.0, ln=False, in_map=False).cuda().eval()
    x = torch.randn(8192, 256, device="cuda")
    lib = nx.load()
    fn = lib.fx_debug_frl_stamps
    fn.argtypes = [ctypes.c_void_p]
    buf = np.zeros(1024 * 8, dtype=np.uint64)
    rows = []
    with torch.no_grad():
        for it in range(6):
            fxf.mstcn(mod, x, T=4096, nvid=2)
            torch.cuda.synchronize()
            assert fn(buf.ctypes.data) == 0
            if it >= 2:
                rows.append(buf.reshape(1024, 8)[:256].astype(np.int64).copy())
    names = ["prologue", "barrier1", "phase1", "epi1", "barrier2", "phase2", "epi2"]
    for st in rows[-2:]:
        t0 = st[:, 0].min()
        print(f"launch: start skew {(st[:, 0].max() - t0) / 100:.2f} us, last stamp {(st[:, 7].max() - t0) / 100:.2f} us, "
              f"first finisher {(st[:, 7].min() - t0) / 100:.2f} us")
        for k, n in enumerate(names):
            d = (st[:, k + 1] - st[:, k]) / 100.0
            print(f"  {n:9s} median {np.median(d):6.2f}  min {d.min():6.2f}  max {d.max():6.2f} us")
        tot = (st[:, 7] - st[:, 0]) / 100.0
        print(f"  {'total':9s} median {np.median(tot):6.2f}  min {tot.min():6.2f}  max {tot.max():6.2f} us")


if __name__ == "__main__":
    main()
