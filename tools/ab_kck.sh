#!/bin/bash
# A/B the training-conv K-chunk cap (VITS_TRAIN_KCK) on the train step (GPU box)
mkdir -p gpurun_out/ab && rm -f gpurun_out/ab/kck_*.log
for r in 1 2; do
  for v in "$@"; do
    VITS_TRAIN_KCK=$v timeout -k 10 300 python3 -u tools/train_bench.py --batch 32 --steps 5 --warmup 2 --graph \
      > gpurun_out/ab/kck_$v.$r.log 2>&1 || exit 1
  done
done
for v in "$@"; do echo "kck=$v $(grep -h utt_per_s gpurun_out/ab/kck_$v.*.log | python3 -c 'import sys,json; print([round(json.loads(l)["s_per_step"]*1e3,2) for l in sys.stdin])')"; done
