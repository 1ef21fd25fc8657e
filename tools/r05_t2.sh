set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_train.py -k "bucketed_rccl" tests/test_train_step_golden.py -k "fp16 or bucketed_rccl" > gpurun_out/r05_t2.txt 2>&1
echo "t2 rc=$?" >> gpurun_out/r05_t2.txt
bash tools/r05_pmc.sh
