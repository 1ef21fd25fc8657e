set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "conv_post" tests/test_models_gpu.py tests/test_configs_gpu.py > gpurun_out/r05_cp_t.txt 2>&1 || exit 1
bash tools/run_longform_profiles.sh r05a > gpurun_out/r05a_lfprof.log 2>&1 || exit 1
echo DONE
