# A/B of the LDS-DMA stream kernel's ring depth x waves per CU on the 1500 B
# config (GPU box only; each cell its own process, the knobs are read once).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/str_sweep.log
for cell in ${CELLS:-3:8 2:8 2:11 4:6 4:8}; do
  r=${cell%%:*}; w=${cell##*:}
  echo "ring=$r wpc=$w" >> gpurun_out/str_sweep.log
  CGCK_STR_RING=$r CGCK_STR_WPC=$w timeout -k 10 120 python tools/sweep.py --variants str,group --workloads 1500 --rounds 3 2>/dev/null | grep median >> gpurun_out/str_sweep.log || exit 1
done
echo done
