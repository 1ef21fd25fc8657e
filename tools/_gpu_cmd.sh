set -e
timeout -k 10 120 python -u tools/stft_ab.py > gpurun_out/r03s_stft_ab.txt 2>&1
VITS_STFT_FWD=0 timeout -k 10 120 python -u tools/stft_ab.py >> gpurun_out/r03s_stft_ab.txt 2>&1
timeout -k 10 200 python -u tools/longform_table.py > gpurun_out/r03s_lf.txt 2>&1
VITS_LOWP_KCK=16 timeout -k 10 200 python -u tools/longform_table.py > gpurun_out/r03s_lf_kc16.txt 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_configs_gpu.py tests/test_infer_bucketed_gpu.py tests/test_models_gpu.py -k "c5 or emovits or lowp or bucketed" > gpurun_out/r03s_tests.txt 2>&1
echo DONE
