"""Summarise a tools/run_profiles.sh run into profiles/<tag>_*.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_summary.json       per-kernel-family time share and, for the
                                    dominant conv kernel, HBM traffic per launch
                                    from the FETCH_SIZE / WRITE_SIZE passes.
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads 1/2 of a wide (16 B/lane) coalesced read stream, so
it is doubled; WRITE_SIZE is exact for 16 B/lane stores (our conv epilogue
stores are 4 B/lane, 128 B-contiguous per half-wave: uncalibrated, used as is).
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
src = os.path.join("gpurun_out", f"prof_{tag}")
dst = "profiles"
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
            os.path.join(dst, f"{tag}_kernel_stats.csv"))

stats = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
total = sum(float(r["TotalDurationNs"]) for r in stats)
fam = defaultdict(lambda: [0, 0.0])
for r in stats:
    name = r["Name"]
    short = name.replace("(anonymous namespace)::", "").replace("void ", "")
    key = ("conv1d_mfma_kernel" if "conv1d_mfma_kernel" in name else
           "resblock_pair_kernel" if any(k in name for k in ("resblock_pair_kernel", "resblock16_kernel",
                                                    "resblock_f32p_kernel")) else
           short.split("(")[0].split("<")[0][:60])
    fam[key][0] += int(r["Calls"])
    fam[key][1] += float(r["TotalDurationNs"])
families = {k: {"calls": v[0], "total_ms": round(v[1] / 1e6, 3),
                "avg_us": round(v[1] / max(1, v[0]) / 1e3, 2),
                "share": round(v[1] / total, 4)} for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])}


def pmc(name):
    rows = list(csv.DictReader(open(os.path.join(src, name, "run_counter_collection.csv"))))
    # the bench's dominant kernel: every conv launch of the step (the conv
    # kernel and the fused ResBlock2 pair kernel)
    vals = [float(r["Counter_Value"]) for r in rows
            if any(k in r["Kernel_Name"] for k in ("conv1d_mfma_kernel", "resblock_pair_kernel",
                                               "resblock16_kernel", "resblock_f32p_kernel"))]
    return vals


fetch = pmc("fetch")
write = pmc("write")
n = min(len(fetch), len(write))
fetch_b = 2.0 * sum(fetch[:n]) * 1024 / n      # gfx950 wide-read correction
write_b = sum(write[:n]) * 1024 / n
summary = {
    "tag": tag,
    "kernel_families": families,
    "conv_kernels": {
        "kernels": "conv1d_mfma_kernel + resblock_pair_kernel + resblock_f32p_kernel",
        "pmc_launches": n,
        "hbm_fetch_bytes_per_launch": round(fetch_b),
        "hbm_write_bytes_per_launch": round(write_b),
        "hbm_bytes_per_launch": round(fetch_b + write_b),
        "note": "FETCH_SIZE x2 (gfx950 wide-read correction), KiB->B; averaged over every conv / fused-pair launch of the infer_p2 steps",
    },
}
with open(os.path.join(dst, f"{tag}_summary.json"), "w") as f:
    json.dump(summary, f, indent=1)
print(json.dumps(summary, indent=1)[:3000])
