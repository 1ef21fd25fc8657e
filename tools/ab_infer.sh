#!/bin/bash
# A/B the headline infer_p2 step under environment settings, interleaved:
#   tools/ab_infer.sh ROUNDS "ENV=a" "ENV=b" ...   -> gpurun_out/ab/infer.<i>.<r>.json
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for e in "$@"; do
    env $e timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-train --no-longform --no-kernels > gpurun_out/ab/infer.$i.$r.json 2> gpurun_out/ab/infer.$i.$r.err || exit 1
    i=$((i+1))
  done
done
echo AB_DONE
