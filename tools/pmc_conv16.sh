#!/bin/bash
# PMC counters for selected conv shapes of tools/conv16_bench.py (GPU box).
export TMPDIR=/tmp
OUT=gpurun_out/pmc_conv16
mkdir -p $OUT
export REPS=2
for shape in "$@"; do
  export ONLY=$shape
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $OUT/$shape/p1 -o run -- python3 tools/conv16_bench.py > $OUT/$shape.p1.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR --output-format csv -d $OUT/$shape/p2 -o run -- python3 tools/conv16_bench.py > $OUT/$shape.p2.log 2>&1 || exit 1
done
echo PMC_DONE
