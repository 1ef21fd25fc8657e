#!/bin/bash
# PMC counters of the weight-gradient kernel on one tools/wgrad_split_bench.py
# shape with fp16 activations (GPU box):  tools/pmc_wgrad.sh "mwd0 k5d5"
export TMPDIR=/tmp IO16=1 ONLY="$1"
OUT=gpurun_out/pmc_wgrad
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $OUT/p1 -o run -- python3 tools/wgrad_split_bench.py > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR --output-format csv -d $OUT/p2 -o run -- python3 tools/wgrad_split_bench.py > $OUT/p2.log 2>&1 || exit 1
for p in p1 p2; do
  f=$(find $OUT/$p -name "*counter_collection.csv" -print -quit)
  python3 - "$f" > $OUT/$p.summary.txt <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "wgrad_kernel" not in r["Kernel_Name"]:
        continue
    acc[(r["Kernel_Name"][:80], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k} {c} n={len(v)} mean={sum(v)/len(v):.4g}")
PY
  rm -rf $OUT/$p
done
echo PMC_DONE
