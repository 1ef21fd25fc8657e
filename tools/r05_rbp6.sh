set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "resblock_pair_f32p" > gpurun_out/r05_rbp6_t.txt 2>&1 || exit 1
ONLY=C128 timeout -k 10 400 python -u tools/rbp_bench.py > gpurun_out/r05_rbp6_b.txt 2>&1
