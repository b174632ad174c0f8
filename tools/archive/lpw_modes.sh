# lpw_kernel (IMIX, packed hint) cost ladder in the lab build: full (the
# deferred 16-byte flush), nodefer (the end-of-chunk flush), noflush, nocons
# (DMA rounds alone), w1 (writer wave); each cell its
# own process, lpw vs slot2 medians on the same buffer (tools/sweep.py imixp).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/lpw_modes.log
export CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/libcgck_lab.so
[ "${CHECK:-1}" = 0 ] || timeout -k 10 300 python tools/lpd_check.py slot2,lpw imix > gpurun_out/lpw_check.log 2>&1 || { tail -n 30 gpurun_out/lpw_check.log; exit 1; }
[ "${CHECK:-1}" = 0 ] || tail -n 1 gpurun_out/lpw_check.log
for m in ${CELLS:-full nodefer noflush full nodefer}; do
  echo "cell $m" >> gpurun_out/lpw_modes.log
  case $m in
  noflush) E="CGCK_LPW_NOFLUSH=1" ;;
  nocons) E="CGCK_LPW_NOCONS=1" ;;
  w1) E="CGCK_LPW_W=1" ;;
  c8) E="CGCK_LPW_C=8" ;;
  nodefer) E="CGCK_LPW_NODEFER=1" ;;
  *) E="CGCK_LPW_X=0" ;;
  esac
  env $E timeout -k 10 120 python tools/sweep.py --variants lpw,slot2 --workloads imixp --rounds ${ROUNDS:-5} > gpurun_out/lpw_cell.log 2>&1 || { cat gpurun_out/lpw_cell.log; exit 1; }
  grep median gpurun_out/lpw_cell.log >> gpurun_out/lpw_modes.log
done
cat gpurun_out/lpw_modes.log
echo done
