#!/bin/bash
# resblock16 store probe (R16_STORE_PROBE: the epilogue computes but does not
# store): what the strided 2-byte output stores cost on the C5 step
# (R16_STORE_PROBE was a temporary store guard in resblock16.hip, removed after this run)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in default r16probe; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lfp_$L -o run -- python3 tools/longform_pmc.py --replays 3 > gpurun_out/lfp_$L.log 2>&1
done
