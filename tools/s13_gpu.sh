#!/bin/bash
# A/B: s_setprio around the MFMA blocks of the global-A conv loop (F32P and 16-bit GA)
WDT=3 bash tools/ab_conv.sh 2 base prio || exit 1
mkdir -p gpurun_out/ab16
for r in 1 2; do for n in base prio; do
  VITS_AMD_LIB=vits_amd/lib/ab_$n.so BF=1 WDT=1 timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/ab16/$n.$r.log 2>&1 || exit 1
done; done
echo S13_DONE
