#!/bin/bash
# kernel trace of the captured train_stft step (R=1 and R=3 replays; per step = diff / 2)
TAG=${1:-s8}
OUT=gpurun_out/tt_$TAG
export TMPDIR=/tmp
mkdir -p $OUT
# one unprofiled run first: MIOpen's find step (its kernels, a first-run-only
# cost kept in the user db) must not land in the R=1 run only - the diff would
# then drop the STFT discriminators' MIOpen convs as "negative"
timeout -k 10 300 python3 tools/train_pmc.py --batch 32 --replays 1 > $OUT/warm.log 2>&1 || exit 1
for R in 1 3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r$R -o run -- \
    python3 tools/train_pmc.py --batch 32 --replays $R > $OUT/r$R.log 2>&1 || exit 1
done
A=$(find $OUT/r1 -name "*kernel_stats.csv" -print -quit)
B=$(find $OUT/r3 -name "*kernel_stats.csv" -print -quit)
python3 tools/train_trace_diff.py "$A" "$B" 2 > gpurun_out/${TAG}_train_kernels.txt
echo TRACE_DONE
