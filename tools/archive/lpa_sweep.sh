# A/B of the lpa kernel's launch shape (blocks per CU) and load policy on the
# 64 B config.  GPU box only; each cell its own process (the knob is read once).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/lpa_sweep.log
for bpc in ${BPCS:-4 8 16}; do
  echo "bpc=$bpc" >> gpurun_out/lpa_sweep.log
  CGCK_LPA_BPC=$bpc timeout -k 10 120 python tools/sweep.py --variants ${VARS:-lpa,90} --workloads 64 --rounds 4 2>/dev/null | grep median >> gpurun_out/lpa_sweep.log || exit 1
done
echo done
