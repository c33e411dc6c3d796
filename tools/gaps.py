"""Diagnostic: idle gaps between kernels in a rocprofv3 kernel trace (last step of a bench run).

python tools/gaps.py <kernel_trace.csv> [steps] [marker]
(marker: a kernel launched once per step, default adam_kernel; combine_kernel without Adam)
"""
import csv
import sys


def main(path, steps=1, marker="adam_kernel"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    # the last `steps` steps: cut at the Adam kernel (end of every step)
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a = ends[-1 - steps] + 1
    b = ends[-1] + 1
    seq = rows[a:b]
    t0, t1 = int(seq[0]["Start_Timestamp"]), int(seq[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seq)
    gaps = [(int(y["Start_Timestamp"]) - int(x["End_Timestamp"]), i) for i, (x, y) in enumerate(zip(seq, seq[1:]))]
    print(f"span {(t1 - t0) / 1e6 / steps:.2f} ms/step  busy {busy / 1e6 / steps:.2f}  kernels {len(seq) / steps:.0f}")
    for lo, hi in ((0, 2e3), (2e3, 5e3), (5e3, 20e3), (20e3, 1e12)):
        sel = [g for g, _ in gaps if lo <= g < hi]
        print(f"  gaps {lo / 1e3:5.0f}-{hi / 1e3:5.0f} us: n {len(sel) / steps:6.0f}  sum {sum(sel) / 1e6 / steps:6.2f} ms")
    print("largest gaps (us): before -> after")
    for g, i in sorted(gaps, reverse=True)[:25]:
        print(f"  {g / 1e3:8.1f}  {seq[i]['Kernel_Name'][:60]} -> {seq[i + 1]['Kernel_Name'][:60]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1, sys.argv[3] if len(sys.argv) > 3 else "adam_kernel")
