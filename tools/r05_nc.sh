set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_train_step_golden.py tests/test_configs_gpu.py > gpurun_out/r05_nc_t.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "
import torch, json, bench
print(json.dumps(bench.kernels_leg(torch.device('cuda:0'))))" > gpurun_out/r05_nc_k.txt 2>&1
