"""Average the rocprofv3 PMC passes of tools/pmc_dominant.sh over the launches of one kernel and
derive its HBM traffic per launch (diagnostic; the JSON it prints is what profiles/pmc_dominant.json
holds and bench.py reports as roofline.traffic).

FETCH_SIZE / WRITE_SIZE are kilobytes per dispatch.  On gfx950 FETCH_SIZE counts 128-B requests of
wide (16 B per lane) reads at 64 B, i.e. half their bytes (MI355X_MICROARCH.md, HBM/rocprofv3), and
every load of this kernel is a 16-B-per-lane global_load_dwordx4, so the fetched bytes are 2 x
FETCH_SIZE; WRITE_SIZE is exact for its 4-B-per-lane stores.
"""
import collections
import csv
import glob
import json
import os
import sys


def main(d, kernel):
    vals = collections.defaultdict(list)
    names = set()
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if kernel not in r["Kernel_Name"]:
                continue
            names.add(r["Kernel_Name"])
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    n = {k: len(v) for k, v in vals.items()}
    out = dict(kernel=kernel, kernel_names=sorted(names), launches_per_counter=n, counters=avg)
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = 2.0 * avg["FETCH_SIZE"] * 1024.0
        write = avg["WRITE_SIZE"] * 1024.0
        out.update(fetch_bytes_per_launch=fetch, write_bytes_per_launch=write,
                   hbm_bytes_per_launch=fetch + write,
                   note="fetch = 2 x FETCH_SIZE (gfx950 wide-read correction), write = WRITE_SIZE; KB -> B")
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        out["stall_split"] = {k: avg[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                          "SQ_WAIT_INST_LDS") if k in avg}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
