"""Per-dispatch device time of ONE replay of the captured C5 step from a
rocprofv3 --kernel-trace csv of tools/longform_pmc.py --replays R (the last
replay: dispatches after the last 'replay' boundary = the last n_per_step).
    python tools/lf_trace_report.py <run_kernel_trace.csv> [label]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
label = sys.argv[2] if len(sys.argv) > 2 else ""
# the replays are identical: the per-step dispatch sequence is the period of
# the tail; find it from the last conv_post (the step's final kernel)
ends = [i for i, r in enumerate(rows) if "conv_post" in r["Kernel_Name"]]
step = rows[ends[-2] + 1:ends[-1] + 1]


def kind(n):
    m = re.search(r"(conv1d_mfma_kernel<[^>]*>|resblock16_kernel\w*?I?Li\d+|resblock_f32p_kernel<[^>]*>|"
                  r"conv_post\w*|\w+_kernel)", n)
    return m.group(1) if m else n[:40]


tot = 0.0
fam = collections.defaultdict(float)
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    g = f'{int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}'
    fam[kind(r["Kernel_Name"])] += d
    print(f"{label} {d:8.1f} us  {g:>12s}  {kind(r['Kernel_Name'])}")
print(f"{label} TOTAL {tot:.1f} us over {len(step)} dispatches")
for k, v in sorted(fam.items(), key=lambda kv: -kv[1]):
    print(f"{label} FAMILY {v:8.1f} us  {k}")
