set -e
timeout -k 10 200 python -u tools/longform_table.py > gpurun_out/r03q_lf_act16.txt 2>&1
VITS_ACT16=0 timeout -k 10 200 python -u tools/longform_table.py > gpurun_out/r03q_lf_act32.txt 2>&1
VITS_GA16=2 timeout -k 10 200 python -u tools/longform_table.py > gpurun_out/r03q_lf_act16_ga.txt 2>&1
DT=fp16 timeout -k 10 200 python -u tools/longform_table.py > gpurun_out/r03q_lf16_act16.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py tests/test_configs_gpu.py tests/test_infer_bucketed_gpu.py > gpurun_out/r03q_tests.txt 2>&1
echo DONE
