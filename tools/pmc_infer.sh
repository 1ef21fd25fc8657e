#!/bin/bash
# PMC counters of every conv / fused-pair dispatch of one infer_p2 step
# (tools/infer_breakdown.py, STEPS=1), two passes (GPU box):
#   p1: effective clock (GRBM_GUI_ACTIVE / 8 / duration), MFMA busy, issue mix
#   p2: wait / active split, LDS conflicts, vector memory instructions
# Report: python tools/pmc_infer_report.py
export TMPDIR=/tmp
OUT=gpurun_out/pmc_infer
mkdir -p $OUT
export STEPS=1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $OUT/p1 -o run -- python3 tools/infer_breakdown.py > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o run -- python3 tools/infer_breakdown.py > $OUT/p2.log 2>&1 || exit 1
echo PMC_INFER_DONE
