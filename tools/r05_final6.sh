set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r05e_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r05e_bench.log 2>&1 || exit 1
bash tools/run_profiles.sh r05e > gpurun_out/r05e_prof.log 2>&1 || exit 1
echo DONE
