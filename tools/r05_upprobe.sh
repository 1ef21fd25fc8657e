#!/bin/bash
# C5 kernel trace with the default library and with the upsampler-store probe
# (UP_STORE_PROBE: the upsample epilogue computes but does not store)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in default upprobe; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lft_$L -o run -- python3 tools/longform_pmc.py --replays 3 > gpurun_out/lft_$L.log 2>&1
done
