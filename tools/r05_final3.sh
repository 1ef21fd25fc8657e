set -o pipefail
mkdir -p gpurun_out
bash tools/run_profiles.sh r05c > gpurun_out/r05c_prof.log 2>&1 || exit 1
bash tools/run_train_profiles.sh r05c 32 > gpurun_out/r05c_trainprof.log 2>&1 || exit 1
bash tools/run_longform_profiles.sh r05c > gpurun_out/r05c_lfprof.log 2>&1 || exit 1
echo DONE
