#!/bin/bash
# A/B of the weight-gradient kernel builds vits_amd/lib/ab_<name>.so on the GPU box
# (tools/wgrad_split_bench.py per build, interleaved ROUNDS times).
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  for n in "$@"; do
    VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 300 python -u tools/wgrad_split_bench.py \
      > gpurun_out/ab/wg_$n.$r.log 2>&1 || exit 1
  done
done
echo AB_DONE
