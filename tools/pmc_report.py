import csv, glob, os, sys
from collections import defaultdict
base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_conv"
for shape in sorted(os.listdir(base)):
    d = os.path.join(base, shape)
    if not os.path.isdir(d):
        continue
    agg = defaultdict(list)
    for p in ("p1", "p2"):
        for f in glob.glob(os.path.join(d, p, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "conv1d_mfma" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    if not m:
        continue
    wc = m.get("SQ_WAVE_CYCLES", 1)
    print(f"== {shape}")
    print("  MFMA busy / GUI_ACTIVE(per XCD*cu?)  mfma_busy=%.3g  gui=%.3g" % (m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0), m.get("GRBM_GUI_ACTIVE", 0)))
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
        print(f"  {k:22s} {m.get(k,0)/wc:6.3f} of wave cycles")
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE"):
        print(f"  {k:22s} {m.get(k,0):.4g}")
