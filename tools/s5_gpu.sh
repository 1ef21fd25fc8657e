#!/bin/bash
# session GPU batch 5: tests on the transposed epilogue, then bench A/B base vs tepi3 (interleaved)
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s5_gputests.log 2>&1 || exit 1
for r in 1 2; do
  for n in base tepi3; do
    VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-kernels > gpurun_out/s5_bench_$n.$r.log 2>&1 || exit 1
  done
done
WDT=1 BF=1 bash tools/ab_conv.sh 1 base tepi3
echo S5_DONE
