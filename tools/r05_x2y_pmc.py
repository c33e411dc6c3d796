"""Per-launch HBM bytes of the X2Y core kernels from tools/r05_x2y_pmc.sh's PMC passes, summed per
bench bracket (fx_prof kinds 3-6): a2f fwd = x2y_a2f_kernel<0>; a2f bwd = x2y_a2f_kernel<1> +
x2y_a2f_dw_kernel; f2a fwd = x2y_f2a_chunk_kernel + x2y_f2a_merge_kernel; f2a bwd = x2y_f2a_bwd_kernel (the
one-launch fused core, the default for calls of >= 64 key chunks) + x2y_f2a_bwd_merge_kernel.  fetch = 2 x FETCH_SIZE (gfx950 wide-read
correction, MI355X_MICROARCH.md), write = WRITE_SIZE; KB -> B."""
import collections
import csv
import glob
import json
import os

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")


def per_kernel(d):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(ROOT, d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def bytes_of(vals, sub):
    tot, n = 0.0, 0
    for name, cs in vals.items():
        if sub in name and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            tot += (2.0 * f + w) * 1024.0
            n += 1
    return tot if n else None


a2f, f2a = per_kernel("pmc_x2y_a2f"), per_kernel("pmc_x2y_f2a")
out = {
    "x2y_a2f_fwd": bytes_of(a2f, "x2y_a2f_kernel<0>"),
    "x2y_a2f_bwd": (lambda a, b: None if a is None else a + (b or 0.0))(bytes_of(a2f, "x2y_a2f_kernel<1>"),
                                                                      bytes_of(a2f, "x2y_a2f_dw_kernel")),
    "x2y_f2a_fwd": (lambda a, b: None if a is None else a + (b or 0.0))(bytes_of(f2a, "x2y_f2a_chunk_kernel"),
                                                                      bytes_of(f2a, "x2y_f2a_merge_kernel")),
    "x2y_f2a_bwd": (lambda a, b: None if a is None else a + (b or 0.0))(bytes_of(f2a, "x2y_f2a_bwd_kernel"),
                                                                      bytes_of(f2a, "x2y_f2a_bwd_merge_kernel")),
    "note": "HBM bytes per launch (fetch = 2 x FETCH_SIZE, write = WRITE_SIZE), kernels of each bench bracket "
            "summed; tools/r05_x2y_bench.py shapes (2 videos x 4096 frames, 32 tokens, head 512)",
}
print(json.dumps(out, indent=1))
