set -o pipefail
mkdir -p gpurun_out
export WDT=3
for r in 1 2; do
timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/r05_ab2_base.$r.txt 2>&1 || exit 1
VITS_AMD_LIB=vits_amd/lib/ab_pre.so timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/r05_ab2_pre.$r.txt 2>&1 || exit 1
done
