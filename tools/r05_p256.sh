#!/bin/bash
# 16-bit 256-channel fused pairs: kernel tests, then the C5 leg per max-k arm
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pair16" > gpurun_out/r05_p256_tests.txt 2>&1
for K in 0 3 7 11 15; do
  timeout -k 10 240 python -u tools/ab_legs.py --legs longform --pair16-256 $K >> gpurun_out/r05_p256_ab.txt 2>&1
done
