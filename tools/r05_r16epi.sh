#!/bin/bash
# resblock16 residual epilogue through LDS (R16_EPI_LDS 1 = the build then, 0 = direct);
# measured slower and removed: "default" in its outputs is the LDS variant
# 16-bit pair / model tests, then the C5 trace and leg per arm
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_models_gpu.py -k "bf16 or f16 or lowp or 16 or c5" > gpurun_out/r05_r16epi_tests.txt 2>&1
for L in default epi0; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lfe_$L -o run -- python3 tools/longform_pmc.py --replays 3 > gpurun_out/lfe_$L.log 2>&1
done
for r in 1 2; do
for L in default epi0; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 240 python -u tools/ab_legs.py --legs longform 2>/dev/null >> gpurun_out/r05_r16epi_ab.txt
done
done
