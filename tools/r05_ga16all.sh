#!/bin/bash
# every inference 16-bit conv group on the GA path (GA16_ALL) vs the k >= 5
# rule: C5 trace + leg per arm, after the 16-bit tests on the variant
# (the GA16_ALL switch in conv1d.hip::ga16 was removed after this measurement)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
VITS_AMD_LIB=vits_amd/lib/ab_ga16all.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_configs_gpu.py tests/test_models_gpu.py -k "bf16 or f16 or lowp or 16 or c5" > gpurun_out/r05_ga16all_tests.txt 2>&1
for L in default ga16all; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lfx_$L -o run -- python3 tools/longform_pmc.py --replays 3 > gpurun_out/lfx_$L.log 2>&1
done
for r in 1 2; do
for L in default ga16all; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 240 python -u tools/ab_legs.py --legs longform 2>/dev/null >> gpurun_out/r05_ga16all_ab.txt
done
done
