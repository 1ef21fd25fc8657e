set -e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stft" > gpurun_out/r03v_stft_tests.txt 2>&1
timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py -k "mrstft" >> gpurun_out/r03v_stft_tests.txt 2>&1
timeout -k 10 120 python -u tools/stft_ab.py > gpurun_out/r03v_stft_ab.txt 2>&1
echo DONE
