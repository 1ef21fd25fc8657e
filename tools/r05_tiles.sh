set -o pipefail
mkdir -p gpurun_out
export WDT=3 TILES=0,3 KCM=1
timeout -k 10 500 python -u tools/conv_bench.py > gpurun_out/r05_tiles_wdt3.txt 2>&1
echo "rc=$?" >> gpurun_out/r05_tiles_wdt3.txt
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_train.py -k "bucketed_rccl" > gpurun_out/r05_t4.txt 2>&1
echo "t4 rc=$?" >> gpurun_out/r05_t4.txt
