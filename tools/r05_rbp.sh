set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "resblock_pair_f32p or generator_fused_pairs" > gpurun_out/r05_rbp_t.txt 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r05_rbp_t.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/rbp_bench.py > gpurun_out/r05_rbp_b.txt 2>&1
echo "rc=$?" >> gpurun_out/r05_rbp_b.txt
