#!/usr/bin/env python
"""Per-(kernel, grid) average durations of a rocprofv3 kernel trace, for the kernels a bench roofline line
times (attention over T, X2Y cores, the fused MS-TCN layer), next to the bench line of the SAME profiled run:
python tools/r06_trace_groups.py <kernel_trace.csv> <bench line json> [out.json]

out.json (committed as profiles/r06_trace_kernels.json): {kernel: {grid size: [launches, average us]}} -- the
kernel-trace durations bench.py divides the roofline_attention / roofline_fused_layer algorithmic bytes and
FLOPs by (`frac`), beside its own live event timing

The bench's roofline entries are on the kernel-time basis (hipExtLaunchKernel event pairs, bench.py Prof);
this prints both so `frac` can be recomputed from the trace (round-5 verdict item 1)."""
import collections
import csv
import json
import sys

KEYS = ("tattn_", "x2y_", "frl_kernel")


def main(trace, bench, out=None):
    rows = list(csv.DictReader(open(trace)))
    grp = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if any(k in n for k in KEYS):
            short = n.replace("fx::(anonymous namespace)::", "").replace("void ", "").replace("fx::", "").split("(")[0]
            grp[(short, int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    print("trace: kernel, grid size, launches, average us")
    for (n, g), d in sorted(grp.items()):
        print(f"  {n:45s} grid {g:8d}  n {len(d):6d}  avg {sum(d) / len(d) / 1e3:8.2f}")
    if out:
        d = collections.defaultdict(dict)
        for (n, g), v in grp.items():
            d[n][str(g)] = [len(v), round(sum(v) / len(v) / 1e3, 3)]
        with open(out, "w") as f:
            json.dump(dict(kernels=d, note="rocprofv3 --kernel-trace of `python bench.py --steps 10 --warmup 3` "
                                          "(tools/r06_diag.sh): per kernel and grid size, [launches, average us]"),
                      f, indent=1, sort_keys=True)
    line = None
    for ln in open(bench):
        ln = ln.strip()
        if ln.startswith("{"):
            line = json.loads(ln)
    if line is None:
        return
    print("bench (same run): kind, kernel us per call, bracket us per call, frac")
    ent = dict(line.get("roofline_attention") or {})
    ent["frl"] = line.get("roofline_fused_layer")
    for k, v in ent.items():
        if not v:
            continue
        if "kernel_ms_per_call" in v:
            print(f"  {k:20s} kernel {1e3 * v['kernel_ms_per_call']:8.2f}  bracket {1e3 * v['bracket_ms_per_call']:8.2f}"
                  f"  kernels/call {v['kernels_per_call']:5.2f}  frac {v['frac']:.4f}  bytes/call {v.get('bytes_per_launch', 0):.4g}")
        else:     # the fused MS-TCN layer: chain-bracket basis, trace cross-check
            print(f"  {k:20s} bracket/launch {1e3 * v['avg_launch_ms']:8.2f}  trace/launch "
                  f"{1e3 * (v.get('trace_avg_launch_ms') or 0):8.2f}  frac {v['frac']:.4f}  trace_frac {v.get('trace_frac')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
