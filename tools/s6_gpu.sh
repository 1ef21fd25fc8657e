#!/bin/bash
# GPU batch 6: STFT-discriminator joined-row layout (first layer default, all layers
# with VITS_STFT_D_HIP_ALL=1): tests, train bench A/B, census; F32P tile/kc sweep
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_train_ops_gpu.py tests/test_mwsd.py tests/test_train_step_golden.py tests/test_configs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s6_tests.log 2>&1 || exit 1
VITS_STFT_D_HIP_ALL=1 $T 400 python -u -m pytest tests/test_mwsd.py tests/test_train_step_golden.py tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s6_tests_all.log 2>&1 || exit 1
$T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s6_bench.log 2>&1 || exit 1
VITS_STFT_D_HIP_ALL=1 $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s6_bench_all.log 2>&1 || exit 1
VITS_STFT_D_HIP_ALL=1 $T 300 python -u tools/train_conv_census.py > gpurun_out/s6_census.log 2>&1 || exit 1
VITS_F32P_KC=16 WDT=3 TILES=0,3 KCM=1,2 $T 400 python -u tools/conv_bench.py > gpurun_out/s6_sweep.log 2>&1
timeout -k 10 200 python -u tools/wn_fallback_debug.py > gpurun_out/s6_wn.log 2>&1
echo S6_DONE
