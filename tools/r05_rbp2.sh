set -o pipefail
mkdir -p gpurun_out
export ONLY=C128
timeout -k 10 200 python -u tools/rbp_bench.py > gpurun_out/r05_rbp2_base.txt 2>&1 || exit 1
VITS_AMD_LIB=vits_amd/lib/ab_p1.so timeout -k 10 200 python -u tools/rbp_bench.py > gpurun_out/r05_rbp2_p1.txt 2>&1
export ONLY=s1.c1 WDT=3
timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/r05_rbp2_kc32.txt 2>&1 || exit 1
F32P_KC=16 timeout -k 10 200 python -u tools/conv_bench.py > gpurun_out/r05_rbp2_kc16.txt 2>&1
