#!/bin/bash
# Where the train_stft step (BASELINE C3/C4) spends its time (run on the GPU box):
# torch.profiler op table + rocprofv3 kernel-trace stats of tools/train_bench.py.
set -e
TAG=${1:-train}
OUT=gpurun_out/prof_$TAG
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/train_bench.py --batch 32 --steps 3 --warmup 2 --graph \
  --torch-prof $OUT/torch_ops.txt > $OUT/train_bench.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 tools/train_bench.py --batch 32 --steps 2 --warmup 1 --graph > $OUT/train_trace.log 2>&1
echo PROF_TRAIN_DONE
