# Same-box A/B of two library builds (con-gen_amd/libcgck_base.so vs the
# current libcgck.so) through tools/sweep.py, interleaved twice.  GPU box only.
# SWEEP_ARGS selects variants/workloads/flags.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ab_lib.log
for i in 1 2; do
  for lib in libcgck_base.so libcgck.so; do
    echo "$lib" >> gpurun_out/ab_lib.log
    CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/$lib timeout -k 10 150 python tools/sweep.py ${SWEEP_ARGS:---variants slot2 --workloads imix --rounds 3} 2>/dev/null | grep median >> gpurun_out/ab_lib.log || exit 1
  done
done
echo done
