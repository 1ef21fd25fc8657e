set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05d_gpu_suite.txt 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r05d_bench.log 2>&1 || exit 1
echo DONE
