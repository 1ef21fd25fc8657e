#!/bin/bash
# A/B the conv kernel builds vits_amd/lib/ab_<name>.so on the GPU box:
# tools/conv_bench.py per build, interleaved ROUNDS times (A B A B ...).
# Usage: tools/ab_conv.sh ROUNDS name1 name2 ...   (env ONLY/BF passed through)
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  for n in "$@"; do
    VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 300 python -u tools/conv_bench.py \
      > gpurun_out/ab/$n.$r.log 2>&1 || exit 1
  done
done
echo AB_DONE
