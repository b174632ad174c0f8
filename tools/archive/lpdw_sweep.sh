# lpd with a writer wave (lpdw_kernel, lab): exactness against lpa and the
# referee on the 64 B shapes (tools/lpd_check.py), then lpa,lpd medians in one
# process per cell, with $CGCK_LPD_W = 0 (lpd_kernel), 16 or 32 (lpdw_kernel).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/lpdw_sweep.log
export CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/libcgck_lab.so
[ "${CHECK:-1}" = 0 ] || CGCK_LPD_W=32 timeout -k 10 300 python tools/lpd_check.py lpa,lpd > gpurun_out/lpdw_check.log 2>&1 || { tail -n 30 gpurun_out/lpdw_check.log; exit 1; }
[ "${CHECK:-1}" = 0 ] || { tail -n 2 gpurun_out/lpdw_check.log; grep -m1 lpdw gpurun_out/lpdw_check.log; }
for w in ${CELLS:-0 32 16 0 32 16}; do
  echo "cell W=$w" >> gpurun_out/lpdw_sweep.log
  CGCK_LPD_W=$w timeout -k 10 120 python tools/sweep.py --variants lpa,lpd --workloads 64 --rounds ${ROUNDS:-5} > gpurun_out/lpdw_cell.log 2>&1 || { cat gpurun_out/lpdw_cell.log; exit 1; }
  grep median gpurun_out/lpdw_cell.log >> gpurun_out/lpdw_sweep.log
done
cat gpurun_out/lpdw_sweep.log
echo done
