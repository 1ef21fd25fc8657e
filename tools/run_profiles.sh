#!/bin/bash
# Collect the rocprofv3 evidence for bench.py's dominant kernel (run on the GPU box).
# 1) kernel trace + stats of the bench command, 2) FETCH_SIZE pass, 3) WRITE_SIZE pass.
set -e
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-train --no-longform --no-kernels > $OUT/bench_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-train --no-longform --no-kernels > $OUT/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-train --no-longform --no-kernels > $OUT/bench_write.log 2>&1
echo PROFILES_DONE
