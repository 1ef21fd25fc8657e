#!/bin/bash
# 16-bit 256-channel pair variants (launch bounds / K chunk) on the C5 leg,
# arms alternated in one call
# (ab libs built by tools/ab_build.sh with EXTRA=-DRP16_OCC...; the
# RP16_OCC / RP16_KC knobs were removed from resblock_f32p.hip after this measurement)
set -e
mkdir -p gpurun_out
for r in 1 2; do
for L in default occ4 kc32 kc32occ4; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 240 python -u tools/ab_legs.py --legs longform --pair16-256 11 2>/dev/null >> gpurun_out/r05_p256b_ab.txt
done
done
