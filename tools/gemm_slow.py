#!/usr/bin/env python
"""Census of the GEMM launches that miss the FAST loaders (FX_GEMM_LOG lines, 14 fields): per shape,
calls and why (A / B not 16-B vectorisable, K not a whole number of 64-deep stages, gathered operand)."""
import collections
import sys

KIND = ["rows", "rconv", "rgen", "cols", "cconv", "rcat", "cconvr", "ckt"]
agg = collections.Counter()
for ln in open(sys.argv[1]):
    f = [int(v) for v in ln.split()]
    if len(f) < 14 or f[11] != 0:
        continue
    M, N, K, b, ak, bk, sp, ca, cb, relu, path, mem, vec, kok = f
    direct = path > 0
    slow = not direct and not ((vec == 3) and (kok or ak == 7) and ak != 2 and bk != 2)
    if slow:
        why = ("A" if not vec & 1 else "") + ("B" if not vec & 2 else "") + ("K" if not kok else "") + \
              ("G" if 2 in (ak, bk) else "")
        agg[(M, N, K, b, KIND[ak], KIND[bk], sp, why)] += 1
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for k, c in agg.most_common(40):
    print(f"{c / steps:7.1f}/step  M {k[0]:6d} N {k[1]:6d} K {k[2]:6d} b {k[3]:3d} {k[4]:>6} x {k[5]:>6} split {k[6]:3d}  {k[7]}")
