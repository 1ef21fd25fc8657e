#!/bin/bash
# PMC HBM traffic + kernel trace of ONE replayed C5 long-form step (GPU box):
# R=1 and R=2 replays, per step = R2 - R1 (tools/summarize_train_profiles.py
# with src prefix prof_<tag>_longform).
set -e
TAG=${1:-r03}
OUT=gpurun_out/prof_${TAG}_longform
export TMPDIR=/tmp
mkdir -p $OUT
for R in 1 2; do
  echo "pass R=$R"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$R -o run -- \
    python3 tools/longform_pmc.py --replays $R > $OUT/trace$R.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch$R -o run -- \
    python3 tools/longform_pmc.py --replays $R > $OUT/fetch$R.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write$R -o run -- \
    python3 tools/longform_pmc.py --replays $R > $OUT/write$R.log 2>&1
done
echo LONGFORM_PROFILES_DONE
