"""Average PMC counters per kernel name over the passes written by tools/pmc_gemm.sh (diagnostic)."""
import collections
import csv
import glob
import os
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "p*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        if os.environ.get("KFILTER", "gemm") not in k:
            continue
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
