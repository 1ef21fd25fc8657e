set -o pipefail
mkdir -p gpurun_out
bash tools/run_longform_profiles.sh r05d > gpurun_out/r05d_lfprof.log 2>&1 || exit 1
echo DONE
