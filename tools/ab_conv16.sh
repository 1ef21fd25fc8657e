#!/bin/bash
# A/B of the io16 training conv between library builds (tools/ab_build.sh),
# interleaved within one GPU call:  tools/ab_conv16.sh ROUNDS name1 name2 ...
#   -> gpurun_out/ab/<name>.<round>.log ; summarise with tools/ab_report.py
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  for n in "$@"; do
    VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 180 python -u tools/conv16_bench.py \
      > gpurun_out/ab/$n.$r.log 2>&1 || { tail -20 gpurun_out/ab/$n.$r.log; exit 1; }
  done
done
python tools/ab_report.py "$@"
