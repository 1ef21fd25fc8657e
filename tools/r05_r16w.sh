set -o pipefail
mkdir -p gpurun_out
VITS_AMD_LIB=vits_amd/lib/ab_wide.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "resblock_pair16 or generator16" > gpurun_out/r05_r16w_t.txt 2>&1 || exit 1
for r in 1 2; do
timeout -k 10 300 python -u tools/ab_legs.py --legs longform 2>>gpurun_out/r05_r16w.err | tail -1 >> gpurun_out/r05_r16w.txt || exit 1
VITS_AMD_LIB=vits_amd/lib/ab_wide.so timeout -k 10 300 python -u tools/ab_legs.py --legs longform 2>>gpurun_out/r05_r16w.err | tail -1 >> gpurun_out/r05_r16w.txt || exit 1
done
VITS_AMD_LIB=vits_amd/lib/ab_wide.so DT=bf16 timeout -k 10 300 python -u tools/longform_table.py > gpurun_out/r05_r16w_table.txt 2>&1
