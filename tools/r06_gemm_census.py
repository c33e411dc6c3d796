"""Round-6 diagnostic: every GEMM of a bench step with its shape and its kernel time.

Run the bench under rocprofv3 with the census build of the library (FACTMX_LIB=.../diag/libfactmx.so, built with
-DFX_GEMM_CENSUS: launch_gemm prints one "GEMM stream M N K batch ak bk split kind persist conv" line per launch),
then join the census lines with the kernel trace in launch order, per stream:
  python tools/r06_gemm_census.py <census stderr> <kernel_trace.csv>
kind: 0 tiled 64x64, 1 direct, 2 wide (128 x 64)."""
import collections
import csv
import sys

GEMM_KEYS = ("gemm_f32_kernel", "gemm_f32_wide8", "gemm_f32_wide_kernel", "gemm_direct_kernel", "gemm_split",
             "gemm_bf16")


def main(census, trace):
    lines = [ln.split()[1:] for ln in open(census) if ln.startswith("GEMM ")]
    by_stream = collections.defaultdict(list)
    for f in lines:
        by_stream[f[0]].append(tuple(int(x) for x in f[1:]))
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Dispatch_Id"]))
    ivs = collections.defaultdict(list)     # per stream: (start, end) of every kernel, for the overlap column
    for r in rows:
        ivs[r["Stream_Id"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))

    def overlap(st, s0, e0):
        """fraction of [s0, e0) during which a kernel of another stream ran"""
        cov = []
        for k, lst in ivs.items():
            if k != st:
                cov += [(max(a, s0), min(b, e0)) for a, b in lst if a < e0 and b > s0]
        cov.sort()
        tot, cur = 0, s0
        for a, b in cov:
            a = max(a, cur)
            if b > a:
                tot += b - a
                cur = b
        return tot / max(e0 - s0, 1)
    kern = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if any(k in n for k in GEMM_KEYS):
            s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            kern[r["Stream_Id"]].append((n.replace("void fx::(anonymous namespace)::", "").split("(")[0],
                                         (e0 - s0) / 1e3, overlap(r["Stream_Id"], s0, e0)))
    # streams matched by launch count (census stream pointer <-> trace stream id)
    cs = sorted(by_stream, key=lambda k: -len(by_stream[k]))
    ts = sorted(kern, key=lambda k: -len(kern[k]))
    agg = collections.defaultdict(lambda: [0, 0.0, "", 0.0])
    for c, t in zip(cs, ts):
        a, b = by_stream[c], kern[t]
        print(f"stream {c}: {len(a)} census lines, trace stream {t}: {len(b)} GEMM kernels", file=sys.stderr)
        for shape, (name, us, ov) in zip(a, b):
            e = agg[(c == cs[0],) + shape]
            e[0] += 1
            e[1] += us
            e[2] = name
            e[3] += ov
    tot = sum(v[1] for v in agg.values())
    print(f"{'stream':6s} {'M':>6} {'N':>5} {'K':>6} {'b':>3} ak bk {'sp':>3} kd {'launch':>6} {'avg us':>8} {'TF/s':>6} {'ovl':>4}  kernel")
    for k, (n, us, name, ov) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        main, M, N, K, b, ak, bk, sp, kind, persist, conv, red = k
        tf = 2.0 * M * N * K * b / (us / n * 1e-6) / 1e12
        print(f"{'main' if main else 'side':6s} {M:6d} {N:5d} {K:6d} {b:3d} {ak:2d} {bk:2d} {sp:3d} {kind:2d} {n:6d} "
              f"{us / n:8.1f} {tf:6.1f} {ov / n:4.2f}  {name[:40]} {'conv' if conv else ''}")
    print(f"total GEMM kernel time {tot / 1e3:.2f} ms over the run")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
