# A/B of the LDS-DMA stream kernels on the 1500 B config, or $WL with $VARS (GPU box only; each
# cell its own process, the knobs are read once).  CELLS: ring:wpc for the
# per-wave form, lcN for the loader/consumer form with N ring phases.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/str_sweep.log
for cell in ${CELLS:-3:8 lc3 lc4}; do
  echo "$cell" >> gpurun_out/str_sweep.log
  case $cell in
  lc*) env CGCK_STR_LC=1 CGCK_STR_LCPH=${cell#lc} timeout -k 10 120 python tools/sweep.py --variants ${VARS:-str,group} --workloads ${WL:-1500} --rounds 3 2>/dev/null | grep median >> gpurun_out/str_sweep.log || exit 1 ;;
  *) env CGCK_STR_RING=${cell%%:*} CGCK_STR_WPC=${cell##*:} timeout -k 10 120 python tools/sweep.py --variants ${VARS:-str,group} --workloads ${WL:-1500} --rounds 3 2>/dev/null | grep median >> gpurun_out/str_sweep.log || exit 1 ;;
  esac
done
echo done
