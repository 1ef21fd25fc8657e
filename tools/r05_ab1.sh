set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_train.py tests/test_train_step_golden.py -k "fp16 or bucketed_rccl" > gpurun_out/r05_t2.txt 2>&1
echo "t2 rc=$?" >> gpurun_out/r05_t2.txt
bash tools/ab_infer.sh 2 "VITS_AMD_LIB=vits_amd/lib/ab_base.so" "VITS_AMD_LIB=vits_amd/lib/ab_xnt.so" "VITS_AMD_LIB=vits_amd/lib/ab_xynt.so" > gpurun_out/r05_ab1.log 2>&1
