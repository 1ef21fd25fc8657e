#!/bin/bash
# A/B of the captured train_stft step under environment settings, interleaved:
#   tools/ab_train.sh ROUNDS "ENV=a" "ENV=b" ...  -> gpurun_out/ab/train.<i>.<r>.log
# (ARGS=... inside a setting adds tools/train_bench.py arguments, e.g.
#  "ARGS=--cudnn-benchmark")
ROUNDS=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for e in "$@"; do
    extra=$(echo "$e" | sed -n 's/.*ARGS=\([^ ]*\).*/\1/p')
    env $(echo "$e" | sed 's/ARGS=[^ ]*//') timeout -k 10 300 python -u tools/train_bench.py \
      --batch 32 --steps 5 --warmup 2 --graph $extra > gpurun_out/ab/train.$i.$r.log 2>&1 || exit 1
    i=$((i+1))
  done
done
echo AB_DONE
