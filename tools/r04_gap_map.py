"""Round-4 diagnostic: main-stream idle gaps of one bench step, in step order (rocprofv3 kernel trace;
step boundary = terms_fwd_kernel).  python tools/r04_gap_map.py <kernel_trace.csv> [min_gap_us]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else 15e3
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Stream_Id'], r['Kernel_Name']) for r in rows)
marks = [s for s, e, st, n in ev if 'terms_fwd_kernel' in n]
main = collections.Counter(st for _, _, st, _ in ev).most_common(1)[0][0]
a, b = marks[-3], marks[-2]
sel = [x for x in ev if a <= x[0] < b and x[2] == main]
prev = None
buck = collections.defaultdict(float)
for s, e, st, n in sel:
    if prev is not None:
        g = s - prev
        if g > 0:
            buck[int((s - a) / 1e6)] += g / 1e3
        if g > thr:
            print(f"t={(s - a) / 1e3:8.1f} us gap {g / 1e3:7.1f} before {n[:80]}")
    prev = e
print("step us", (b - a) / 1e3, "gap us per ms of step:", {k: round(v) for k, v in sorted(buck.items())})
