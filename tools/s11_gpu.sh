#!/bin/bash
# full GPU suite on the final tree, MR-STFT kernel timing, final bench line
T="timeout -k 10"
$T 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s11_tests.log 2>&1 || exit 1
$T 200 python -u tools/stft_ab.py > gpurun_out/s11_stft.log 2>&1 || exit 1
VITS_STFT_FWD=1 $T 420 python -u bench.py > gpurun_out/r03c_bench.log 2>&1
echo S11_DONE
