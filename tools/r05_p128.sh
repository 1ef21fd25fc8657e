#!/bin/bash
# 16-bit 128-channel pairs through resblock_f32p's streamed-K tile (ab libs):
# parity of the routed kernel, then the C5 leg per arm, alternated
# (ab libs built by tools/ab_build.sh with EXTRA=-DRP16_ROUTE128...; the
# RP16_ROUTE128 / RP16_KC128 / RP16_OCC128 knobs were removed from resblock_f32p.hip after this measurement)
set -e
mkdir -p gpurun_out
VITS_AMD_LIB=vits_amd/lib/ab_r128.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pair16_fused and 128" > gpurun_out/r05_p128_tests.txt 2>&1
for r in 1 2; do
for L in default r128 r128kc64 r128occ4; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 240 python -u tools/ab_legs.py --legs longform 2>/dev/null >> gpurun_out/r05_p128_ab.txt
done
done
