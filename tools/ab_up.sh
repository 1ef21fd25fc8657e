#!/bin/bash
# A/B of conv builds on the upsampler / decoder shapes + the infer step breakdown
mkdir -p gpurun_out/ab && rm -f gpurun_out/ab/*.log
for r in 1 2; do
  for n in "$@"; do
    VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/ab/$n.$r.log 2>&1 || exit 1
  done
done
for n in "$@"; do
  VITS_AMD_LIB=vits_amd/lib/ab_$n.so STEPS=5 timeout -k 10 200 python -u tools/infer_breakdown.py > gpurun_out/ab/bd_$n.log 2>&1 || exit 1
done
echo AB_DONE
