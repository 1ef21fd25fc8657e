#!/bin/bash
# session-4 GPU batch: transposed-epilogue A/B, F32P tile/kc sweep, training conv census
set -e
WDT=3 bash tools/ab_conv.sh 2 base tepi2
VITS_AMD_LIB=vits_amd/lib/ab_tepi2.so WDT=3 TILES=0,3 timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/s4_sweep_kc32.log 2>&1
VITS_AMD_LIB=vits_amd/lib/ab_tepi2.so VITS_F32P_KC=16 WDT=3 TILES=0,3 timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/s4_sweep_kc16.log 2>&1
timeout -k 10 300 python -u tools/train_conv_census.py > gpurun_out/s4_census.log 2>&1
echo S4_DONE
