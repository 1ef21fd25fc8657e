set -e
bash tools/run_profiles.sh r03
bash tools/run_longform_profiles.sh r03
timeout -k 10 300 python -u tools/train_op_stacks.py > gpurun_out/r03x_op_stacks.txt 2>&1
echo DONE
