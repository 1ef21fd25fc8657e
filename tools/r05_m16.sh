set -o pipefail
mkdir -p gpurun_out/ab
export WDT=3
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_configs_gpu.py > gpurun_out/r05_m16_tests.txt 2>&1
echo "tests rc=$?" >> gpurun_out/r05_m16_tests.txt
for n in base m16; do
  VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/ab/conv_$n.log 2>&1 || exit 1
done
bash tools/ab_infer.sh 2 "VITS_AMD_LIB=vits_amd/lib/ab_base.so" "VITS_AMD_LIB=vits_amd/lib/ab_m16.so" > gpurun_out/r05_ab_m16.log 2>&1
