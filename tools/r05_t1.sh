set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -v -s --timeout 400 --timeout-method thread tests/ > gpurun_out/r05_t1_gpu.txt 2>&1
echo "gpu suite rc=$?" >> gpurun_out/r05_t1_gpu.txt
