set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/glue_sites.py > gpurun_out/r05_glue_sites.txt 2>&1 || exit 1
bash tools/train_trace.sh r05a > gpurun_out/r05_trace.log 2>&1
