#!/bin/bash
# GPU batch 7: full GPU suite; all-layer HIP STFT discriminator (V4 rows) A/B on the train legs
T="timeout -k 10"
$T 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s7_gputests.log 2>&1 || exit 1
VITS_STFT_D_HIP_ALL=1 $T 300 python -u -m pytest tests/test_mwsd.py tests/test_train_step_golden.py tests/test_train.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s7_tests_all.log 2>&1 || exit 1
$T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s7_bench.log 2>&1 || exit 1
VITS_STFT_D_HIP_ALL=1 $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s7_bench_all.log 2>&1 || exit 1
$T 200 python -u tools/wn_fallback_debug.py > gpurun_out/s7_wn.log 2>&1
echo S7_DONE
