mkdir -p gpurun_out/ab && rm -f gpurun_out/ab/*.log
for r in 1 2; do
  for n in base noprio occ4 occ2; do
    occ=""; [ $n = occ4 ] && occ="1:4"; [ $n = occ2 ] && occ="1:2"
    VITS_TILE_OCC=$occ VITS_AMD_LIB=vits_amd/lib/ab_$n.so timeout -k 10 300 python -u tools/conv_bench.py > gpurun_out/ab/$n.$r.log 2>&1 || exit 1
  done
done
echo AB_DONE
