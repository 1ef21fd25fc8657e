#!/bin/bash
# paired real-input MR-STFT forward: parity tests, then A/B vs the unpaired build
T="timeout -k 10"
$T 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s10_tests.log 2>&1 || exit 1
for r in 1 2; do
  for n in nopair main; do
    if [ $n = main ]; then L=vits_amd/lib/libvits_amd.so; else L=vits_amd/lib/ab_$n.so; fi
    VITS_AMD_LIB=$L $T 200 python -u tools/stft_ab.py > gpurun_out/s10_stft_$n.$r.log 2>&1 || exit 1
  done
done
timeout -k 10 420 python -u bench.py > gpurun_out/r03c_bench.log 2>&1
echo S10_DONE
