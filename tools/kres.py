#!/usr/bin/env python
"""Per-kernel register / scratch / LDS usage of one HIP source for gfx950 (hipcc's
kernel-resource-usage remarks), as a table: python tools/kres.py fact-clip_amd/csrc/gemm_f32.hip [filter]."""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Iinclude", "-c", src, "-o", "/tmp/_kres.o",
       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*)", line)
    if not m:
        continue
    t = re.sub(r"\s*\[-Rpass-analysis=.*\]$", "", m.group(1)).strip()
    if t.startswith("Function Name:"):
        cur = {"name": re.sub(r"^_ZN2fx12_GLOBAL__N_1\d+", "", t.split(":", 1)[1].strip())}
        rows.append(cur)
    elif cur is not None:
        for key, short in (("VGPRs", "VGPRs"), ("AGPRs", "AGPRs"), ("ScratchSize [bytes/lane]", "ScratchSize"),
                           ("LDS Size [bytes/block]", "LDS"), ("Occupancy [waves/SIMD]", "Occupancy"),
                           ("VGPRs Spill", "Spill")):
            if t.startswith(key + ":"):
                cur[short] = t.split(":", 1)[1].strip()
seen = set()
for r in rows:
    if flt not in r["name"] or r["name"] in seen:
        continue
    seen.add(r["name"])
    print(f"{r['name'][:70]:70s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>4} "
          f"scratch {r.get('ScratchSize', '?'):>4} spill {r.get('Spill', '?'):>3} lds {r.get('LDS', '?'):>6} occ {r.get('Occupancy', '?')}")
