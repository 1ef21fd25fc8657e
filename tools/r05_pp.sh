set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_ops_gpu.py tests/test_train_step_golden.py tests/test_wnorm_gpu.py tests/test_train.py > gpurun_out/r05_pp_t.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/pack_census.py > gpurun_out/r05_pack_census.txt 2>&1
timeout -k 10 300 python -u tools/ab_legs.py --legs train > gpurun_out/r05_pp_train.txt 2>&1
