#!/usr/bin/env python
"""Where one training step's time goes, from a rocprofv3 kernel trace (round 5).

python tools/step_map.py <kernel_trace.csv> [steps]

Step boundary: the loss-table forward kernel (terms_fwd_kernel), one per step.  Over the last `steps`
complete steps: wall time per step, launches per step and stream, per kernel category the kernel time
on the main stream and on the others, and the DEVICE-idle time (no kernel of this process running on
any stream) split by what the main stream launched next -- the host-bound stretches."""
import collections
import csv
import sys

CATS = [  # (category, substrings of the kernel name), first match wins
    ("frl (fused MS-TCN layer)", ["frl_kernel"]),
    ("token decoder kernel", ["tok_kernel"]),
    ("gru", ["gru_fwd", "gru_bwd"]),
    ("attention over T", ["tattn_"]),
    ("x2y cores", ["x2y_"]),
    ("small MHA", ["mha_small"]),
    ("direct GEMM (token rows)", ["gemm_direct"]),
    ("frame GEMM wide8", ["gemm_f32_wide8", "gemm_f32_wide_kernel", "gemm_bf16", "gemm_split"]),
    ("tiled GEMM 64x64", ["gemm_f32_kernel"]),
    ("split-K reduce", ["splitk_reduce"]),
    ("LayerNorm", ["ln_fwd", "ln_bwd", "ln_param"]),
    ("loss / eval (vloss)", ["terms_", "match_cost", "eval_pred", "combine", "infonce"]),
    ("segments / pooling", ["seg_", "argmax", "boundary"]),
    ("adam / norm", ["adam", "sumsq", "norm_final"]),
    ("weight packing", ["pack_"]),
    ("dropout", ["dropout_kernel"]),
    ("rowops (softmax/pf/l2/relu/add)", ["softmax", "pf_", "l2n", "relu_bwd", "add2", "colsum", "rowscat"]),
    ("torch / copies", ["at::", "rocclr", "copyBuffer", "fillBuffer"]),
]


def cat(name):
    for c, keys in CATS:
        if any(k in name for k in keys):
            return c
    return "other"


def main(path, nsteps):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    marks = [s for s, e, st, n in ev if "terms_fwd_kernel" in n]
    main_st = collections.Counter(st for _, _, st, _ in ev).most_common(1)[0][0]
    nsteps = min(nsteps, len(marks) - 1)
    a, b = marks[-1 - nsteps], marks[-1]
    sel = [x for x in ev if a <= x[0] < b]
    per = float(nsteps)
    wall = (b - a) / 1e6 / per
    launches = collections.Counter("main" if st == main_st else "other" for _, _, st, _ in sel)
    t_cat = collections.defaultdict(lambda: [0.0, 0.0, 0])
    for s, e, st, n in sel:
        c = t_cat[cat(n)]
        c[0 if st == main_st else 1] += (e - s) / 1e3
        c[2] += 1
    # device-idle intervals: union of all kernel intervals
    idle = collections.defaultdict(float)
    idle_total = 0.0
    cover = a
    for s, e, st, n in sel:
        if s > cover:
            g = (s - cover) / 1e3
            idle_total += g
            idle[cat(n)] += g
        cover = max(cover, e)
    main_busy = sum((e - s) for s, e, st, n in sel if st == main_st) / 1e3
    print(f"{nsteps} steps: wall {wall:.3f} ms/step, launches/step main {launches['main'] / per:.0f} "
          f"other {launches['other'] / per:.0f}; main-stream kernel time {main_busy / 1e3 / per:.3f} ms; "
          f"device idle {idle_total / 1e3 / per:.3f} ms/step")
    print(f"{'category':34s} {'main ms':>8} {'other ms':>9} {'launch':>7} {'idle-before ms':>15}")
    for c in sorted(t_cat, key=lambda k: -(t_cat[k][0] + t_cat[k][1])):
        m, o, n = t_cat[c]
        print(f"{c:34s} {m / 1e3 / per:8.3f} {o / 1e3 / per:9.3f} {n / per:7.1f} {idle[c] / 1e3 / per:15.3f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
