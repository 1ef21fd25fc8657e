#!/bin/bash
# PMC HBM traffic + kernel trace of ONE captured train_stft step (run on the GPU box).
# Each quantity is measured with R=1 and R=2 replays; per step = R2 - R1.
set -e
TAG=${1:-r03}
B=${2:-32}
OUT=gpurun_out/prof_${TAG}_train
export TMPDIR=/tmp
mkdir -p $OUT
# one unprofiled run first: MIOpen's exhaustive find (cudnn.benchmark, as the
# bench) writes the box's find-db, so every profiled run below starts from
# the same db and R=2 - R=1 cancels the search
timeout -k 10 300 python3 tools/train_pmc.py --batch $B --replays 1 > $OUT/warm.log 2>&1
for R in 1 2; do
  echo "pass R=$R"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$R -o run -- \
    python3 tools/train_pmc.py --batch $B --replays $R > $OUT/trace$R.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch$R -o run -- \
    python3 tools/train_pmc.py --batch $B --replays $R > $OUT/fetch$R.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write$R -o run -- \
    python3 tools/train_pmc.py --batch $B --replays $R > $OUT/write$R.log 2>&1
done
echo TRAIN_PROFILES_DONE
