#!/bin/bash
# upsampler output tile staged through LDS (UP_LDS 1 = default build) vs the
# per-element strided stores (ab_uplds0): GPU suite on the default build, C5
# trace per arm, then the headline (no train / long-form / kernels legs) and
# the C5 leg, arms alternated
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_uplds_suite.txt 2>&1
for L in default uplds0; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lfu_$L -o run -- python3 tools/longform_pmc.py --replays 3 > gpurun_out/lfu_$L.log 2>&1
done
for r in 1 2; do
for L in default uplds0; do
  if [ $L = default ]; then unset VITS_AMD_LIB; else export VITS_AMD_LIB=vits_amd/lib/ab_$L.so; fi
  timeout -k 10 300 python -u bench.py --no-train --no-longform --no-kernels --no-cpu-baseline --no-roofline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$L headline', d['ms_per_step'])" >> gpurun_out/r05_uplds_ab.txt
  timeout -k 10 240 python -u tools/ab_legs.py --legs longform 2>/dev/null >> gpurun_out/r05_uplds_ab.txt
done
done
