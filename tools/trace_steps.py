"""Diagnostic: per-step main/side stream busy time and main-stream idle gaps from a rocprofv3
kernel trace of bench.py (step boundary = the terms_fwd_kernel launch, one per step)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Stream_Id'], r['Kernel_Name']) for r in rows)
marks = [s for s, e, st, n in ev if 'terms_fwd_kernel' in n]
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 10
main = collections.Counter(st for _, _, st, _ in ev).most_common(1)[0][0]
for i in range(len(marks) - nlast, len(marks) - 1):
    a, b = marks[i], marks[i + 1]
    sel = [x for x in ev if a <= x[0] < b]
    busy = collections.defaultdict(int)
    for s, e, st, n in sel:
        busy[st] += e - s
    m = [x for x in sel if x[2] == main]
    gaps = [m[j + 1][0] - m[j][1] for j in range(len(m) - 1)]
    big = sorted(((g, m[j][3][:60], m[j + 1][3][:60]) for j, g in enumerate(gaps)), reverse=True)[:int(sys.argv[3]) if len(sys.argv) > 3 else 0]
    print(f"step {(b - a) / 1e3:8.1f} us  main busy {busy[main] / 1e3:8.1f}  other {sum(v for k, v in busy.items() if k != main) / 1e3:8.1f}"
          f"  main launches {len(m)}  gaps>0 sum {sum(g for g in gaps if g > 0) / 1e3:7.1f} us")
    for g in big:
        print(f"     gap {g[0] / 1e3:7.1f} us after {g[1]} before {g[2]}")
