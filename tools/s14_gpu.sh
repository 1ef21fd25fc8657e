#!/bin/bash
# HIP training LayerNorm: full GPU suite, then train legs A/B vs torch's layer_norm
T="timeout -k 10"
$T 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s14_tests.log 2>&1 || exit 1
for r in 1 2; do
  $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s14_bench_hip.$r.log 2>&1 || exit 1
  VITS_LN_HIP=0 $T 300 python -u bench.py --no-cpu-baseline --no-kernels --no-longform > gpurun_out/s14_bench_torch.$r.log 2>&1 || exit 1
done
echo S14_DONE
