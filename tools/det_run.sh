set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/determinism.py 3 > gpurun_out/r05_det_hip.txt 2>&1 &&
MODE=torch DET=1 timeout -k 10 300 python -u tools/determinism.py 3 > gpurun_out/r05_det_torch.txt 2>&1 &&
DET=1 timeout -k 10 300 python -u tools/determinism.py 2 > gpurun_out/r05_det_hip_det.txt 2>&1
