set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
VITS_AMD_LIB=vits_amd/lib/ab_old.so timeout -k 10 300 python -u tools/ab_legs.py --xb16 6144 2>>gpurun_out/r05_ab3.err | tail -1 >> gpurun_out/r05_ab3.txt || exit 1
timeout -k 10 300 python -u tools/ab_legs.py --xb16 6144 2>>gpurun_out/r05_ab3.err | tail -1 >> gpurun_out/r05_ab3.txt || exit 1
timeout -k 10 300 python -u tools/ab_legs.py 2>>gpurun_out/r05_ab3.err | tail -1 >> gpurun_out/r05_ab3.txt || exit 1
done
