"""Per-step kernel breakdown of a graph-replayed train step from a rocprofv3
kernel trace (tools/prof_train.sh): the replays are the final run of
back-to-back dispatches; one step = that run / REPLAYS."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_train_r02/trace/run_kernel_trace.csv"
replays = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
segs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) > 2e6:
        segs.append(cur)
        cur = []
    cur.append(b)
segs.append(cur)
last = segs[-1]
n = len(last) // replays
step = last[-n:]
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step) / 1e6
print(f"{n} dispatches per step, {wall:.2f} ms wall, {busy:.2f} ms in kernels")
fam = defaultdict(lambda: [0, 0.0])
for r in step:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    if name.startswith("at::native::"):
        name = name[12:]
    key = name.split("(")[0][:110]
    fam[key][0] += 1
    fam[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
small = sum(1 for r in step if int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) < 8000)
print(f"dispatches under 8 us: {small}")
for k, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{t:8.3f} ms {c:5d} {t / c * 1e3:8.1f} us  {k}")
