"""Per-dispatch report of tools/pmc_infer.sh: for the conv / fused-pair
dispatches of the profiled infer_p2 step, the effective shader clock
(GRBM_GUI_ACTIVE is summed over the 8 XCDs: clock = GUI / 8 / duration,
MI355X_MICROARCH.md DVFS note), MFMA-pipe utilisation (SQ_VALU_MFMA_BUSY_CYCLES
summed over the 1024 SIMDs / (1024 * GUI / 8)), and issue mix per MFMA."""
import csv
import glob
import os
import sys
from collections import defaultdict

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_infer"
KEYS = ("conv1d_mfma_kernel", "resblock_pair_kernel")


def load(p):
    rows = defaultdict(dict)
    meta = {}
    for f in glob.glob(os.path.join(base, p, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if not any(k in r["Kernel_Name"] for k in KEYS):
                continue
            d = int(r["Dispatch_Id"])
            rows[d][r["Counter_Name"]] = float(r["Counter_Value"])
            meta[d] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                       int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"]))
    return rows, meta


p1, m1 = load("p1")
p2, m2 = load("p2")
# the last step's launches (81 conv / pair launches per infer_p2 step)
last = int(os.environ.get("LAST", "81"))
d1, d2 = sorted(p1)[-last:], sorted(p2)[-last:]
n = min(len(d1), len(d2))
print(f"{'#':>3} {'us':>8} {'GHz':>5} {'mfma%':>6} {'valu/mf':>7} {'salu/mf':>7} {'lds/mf':>6} "
      f"{'wait':>5} {'winst':>5} {'vgpr':>4} {'lds':>6}  kernel")
tot_t = tot_busy = tot_gui = 0.0
for i in range(n):
    a, b = p1[d1[i]], p2[d2[i]]
    name, dur, vg, ag, lds = m1[d1[i]]
    gui = a.get("GRBM_GUI_ACTIVE", 0) / 8
    clk = gui / dur if dur else 0
    mf = a.get("SQ_INSTS_MFMA", 0)
    util = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (1024 * gui) if gui else 0
    wc = a.get("SQ_WAVE_CYCLES", 1)
    short = name.split("<")[0].split("::")[-1] + "<" + name.split("<", 1)[1].split(">")[0] + ">" if "<" in name else name
    print(f"{i:3d} {dur / 1e3:8.1f} {clk:5.2f} {util * 100:6.1f} {a.get('SQ_INSTS_VALU', 0) / max(mf, 1):7.2f} "
          f"{a.get('SQ_INSTS_SALU', 0) / max(mf, 1):7.2f} {a.get('SQ_INSTS_LDS', 0) / max(mf, 1):6.2f} "
          f"{a.get('SQ_WAIT_ANY', 0) / wc:5.2f} {b.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} {vg + ag:4d} {lds:6d}  {short[:60]}")
    tot_t += dur
    tot_busy += a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    tot_gui += gui
print(f"total {tot_t / 1e6:.3f} ms, time-weighted clock {tot_gui / tot_t:.2f} GHz, "
      f"MFMA util {tot_busy / (1024 * tot_gui) * 100:.1f} %")
