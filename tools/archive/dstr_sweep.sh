# dstr_kernel (cgck_dense.hip) on the 1500 B config: exactness against the
# group kernel and the referee (tools/lpd_check.py mtu), then in-process A/B
# medians against group for each cell D:C:WPC (GPU box only; each cell its
# own process, the knobs are read once).  CELLS: D:C:WPC[:MODE[:W[:F]]]; CHECK=0 skips
# the exactness pass.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/dstr_sweep.log
export CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/libcgck_lab.so
[ "${CHECK:-1}" = 0 ] || CGCK_DSTR_F=${CHECKF:-0} timeout -k 10 300 python tools/lpd_check.py group,dstr mtu > gpurun_out/dstr_check.log 2>&1 || { tail -n 30 gpurun_out/dstr_check.log; exit 1; }
tail -n 1 gpurun_out/dstr_check.log
for cell in ${CELLS:-3:16:8 2:16:8 3:8:8 3:32:8 3:64:8 2:32:12}; do
  IFS=: read d c w m wr f <<< "$cell"
  echo "cell D=$d C=$c WPC=$w MODE=${m:-0} W=${wr:-1} F=${f:-0}" >> gpurun_out/dstr_sweep.log
  env CGCK_DSTR_D=$d CGCK_DSTR_C=$c CGCK_DSTR_WPC=$w CGCK_DSTR_MODE=${m:-0} CGCK_DSTR_W=${wr:-1} CGCK_DSTR_F=${f:-0} timeout -k 10 120 python tools/sweep.py --variants ${VARS:-group,dstr} --workloads ${WL:-1500} --rounds ${ROUNDS:-3} > gpurun_out/dstr_cell.log 2>&1 || { cat gpurun_out/dstr_cell.log; exit 1; }
  grep median gpurun_out/dstr_cell.log >> gpurun_out/dstr_sweep.log
done
cat gpurun_out/dstr_sweep.log
echo done
