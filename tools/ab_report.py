"""Summarise tools/ab_conv.sh logs: per shape, the best TF/s of each build
over the rounds, and the total conv time (min over rounds)."""
import glob
import os
import re
import sys
from collections import defaultdict

names = sys.argv[1:]
res = defaultdict(lambda: defaultdict(list))
tot = defaultdict(list)
for n in names:
    for f in sorted(glob.glob(f"gpurun_out/ab/{n}.*.log")):
        for line in open(f):
            m = re.match(r"^(\S+)\s+cin=.*\s([\d.]+) TF/s", line)
            if m:
                res[m.group(1)][n].append(float(m.group(2)))
            m = re.match(r"TOTAL ([\d.]+) TF/s over ([\d.]+) ms", line)
            if m:
                tot[n].append(float(m.group(2)))
print(f"{'shape':18s}" + "".join(f"{n:>10s}" for n in names))
for shape, d in res.items():
    print(f"{shape:18s}" + "".join(f"{max(d[n]) if d[n] else 0:10.1f}" for n in names))
print(f"{'TOTAL ms (min)':18s}" + "".join(f"{min(tot[n]) if tot[n] else 0:10.2f}" for n in names))
print(f"{'TOTAL ms (all)':18s}" + "  ".join(",".join(f"{v:.2f}" for v in tot[n]) for n in names))
