"""Join the FX_GEMM_LOG shape log with a rocprofv3 kernel trace: time per GEMM shape (diagnostic).

python tools/gemm_census.py <gemm_log> <kernel_trace.csv>
"""
import collections
import csv
import sys

KIND = ["rows", "rconv", "rgen", "cols", "cconv", "rcat"]


def main(log_path, trace_path):
    # one kernel per log line, except the members > 0 of a grouped launch (12th field), which share
    # the kernel of the line before: their time is booked to the group's first line
    shapes = [tuple(int(v) for v in ln.split()) for ln in open(log_path) if ln.strip()]
    shapes = [sh for sh in shapes if len(sh) < 12 or sh[11] == 0]
    rows = sorted(csv.DictReader(open(trace_path)), key=lambda r: int(r["Start_Timestamp"]))
    g = [r for r in rows if "gemm_f32_kernel" in r["Kernel_Name"] or "gemm_f32_wide" in r["Kernel_Name"] or "gemm_direct_kernel" in r["Kernel_Name"] or "gemm_direct_group" in r["Kernel_Name"]]
    red = [r for r in rows if "splitk_reduce" in r["Kernel_Name"]]
    n = min(len(g), len(shapes))
    g, shapes = g[-n:], shapes[-n:]
    agg = collections.defaultdict(lambda: [0, 0.0])
    for s, r in zip(shapes, g):
        key = s[:7] + (s[10] if len(s) > 10 else -1,)
        agg[key][0] += 1
        agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{n} gemm launches, {tot/1e3:.2f} ms; split-K reduces: {len(red)}")
    print(f"{'M':>6} {'N':>6} {'K':>6} {'b':>3} {'A':>5} {'B':>5} {'sp':>3} {'dw':>3} {'calls':>6} {'avg us':>8} {'tot ms':>8} {'TF/s':>7}")
    for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
        M, N, K, b, ak, bk, sp, dw = k
        tf = 2.0 * M * N * K * b / (us / c * 1e-6) / 1e12
        print(f"{M:6d} {N:6d} {K:6d} {b:3d} {KIND[ak]:>5} {KIND[bk]:>5} {sp:3d} {dw:3d} {c:6d} {us/c:8.1f} {us/1e3:8.2f} {tf:7.1f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
