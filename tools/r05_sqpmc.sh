#!/bin/bash
# SQ stall breakdown of the captured C5 step (one replay) per kernel:
# wave cycles split into parked (s_waitcnt / barrier), issue-stalled and
# active, MFMA busy cycles, LDS bank conflicts; GRBM_GUI_ACTIVE for the clock
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/sqpmc -o run -- python3 tools/longform_pmc.py --replays 1 > gpurun_out/sqpmc.log 2>&1
