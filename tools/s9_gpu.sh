#!/bin/bash
# all-layer HIP STFT discriminator (4-step-padded joined rows) vs MIOpen layers: train legs A/B + per-step trace
T="timeout -k 10"
for r in 1 2; do
  $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s9_bench_def.$r.log 2>&1 || exit 1
  VITS_STFT_D_HIP_ALL=1 $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s9_bench_all.$r.log 2>&1 || exit 1
done
for r in 1 2; do VITS_TRAIN_GEMM1X1=256 $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s9_bench_gemm.$r.log 2>&1 || exit 1; done
VITS_TRAIN_GEMM1X1=256 $T 300 python -u -m pytest tests/test_train_step_golden.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s9_tests_gemm.log 2>&1
echo S9_DONE
