set -o pipefail
export WDT=3
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/conv_bench.py > gpurun_out/r05_convbench_wdt3.txt 2>&1 &&
timeout -k 10 600 bash tools/pmc_conv.sh s1.c1.k11d1 s1.c1.k3d1 s1.c2.k3 s1.c2.k11 s0.c1.k7d3 flow.in > gpurun_out/r05_pmc.log 2>&1
