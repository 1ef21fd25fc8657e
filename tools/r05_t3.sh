set -o pipefail
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-result -o /tmp/mfma_probe tools/mfma_probe.hip &&
timeout -k 10 120 /tmp/mfma_probe > gpurun_out/r05_mfma_probe.txt 2>&1
echo "probe rc=$?" >> gpurun_out/r05_mfma_probe.txt
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_train.py tests/test_train_step_golden.py -k "fp16_autocast_vs or bucketed_rccl" > gpurun_out/r05_t3.txt 2>&1
echo "t3 rc=$?" >> gpurun_out/r05_t3.txt
