#!/bin/bash
# end-of-session evidence: full bench line, headline kernel trace + PMC traffic, train-step trace + PMC traffic
TAG=${1:-r03b}
timeout -k 10 420 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
bash tools/run_profiles.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
bash tools/run_train_profiles.sh $TAG 32 > gpurun_out/${TAG}_trainprof.log 2>&1 || exit 1
echo FINAL_DONE
