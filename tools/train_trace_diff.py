"""Per-step kernel table of the captured train_stft step: two rocprofv3
--kernel-trace --stats runs of tools/train_pmc.py with R=1 and R=1+N replays;
(stats_b - stats_a) / N per kernel = one replayed step (eager warm-up and the
capture cancel).  python tools/train_trace_diff.py A_stats.csv B_stats.csv N"""
import csv
import sys


def load(p):
    out = {}
    with open(p) as f:
        for r in csv.DictReader(f):
            out[r["Name"]] = (int(r["Calls"]), float(r["TotalDurationNs"]))
    return out


a, b, n = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3])
rows = []
for k, (cb, tb) in b.items():
    ca, ta = a.get(k, (0, 0.0))
    if cb - ca > 0:
        rows.append(((tb - ta) / n / 1e6, (cb - ca) / n, k))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"per step: {tot:.3f} ms kernel time, {sum(r[1] for r in rows):.0f} dispatches")
for ms, c, k in rows[:60]:
    print(f"{ms:8.3f} ms {c:6.0f}x  {k[:150]}")
