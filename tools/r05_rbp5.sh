set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_configs_gpu.py tests/test_infer_bucketed_gpu.py > gpurun_out/r05_rbp5_t.txt 2>&1 || exit 1
EXTRA="no32=64:11,128:7,256:3" timeout -k 10 400 python -u tools/ab_pairs.py > gpurun_out/r05_abpairs3.txt 2>&1
