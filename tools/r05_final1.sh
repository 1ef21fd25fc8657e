set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/r05a_bench.log 2>&1 || exit 1
bash tools/run_profiles.sh r05a > gpurun_out/r05a_prof.log 2>&1 || exit 1
echo DONE
