# Same-box A/B of library builds (con-gen_amd/libcgck_base.so vs the
# current libcgck.so, or $LIBS) through tools/sweep.py, interleaved $REPS
# times (default 2).  GPU box only.  SWEEP_ARGS selects variants/workloads/
# flags; RSS=1 adds tools/rss_bench.py (the batched Toeplitz hash).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/ab_lib.log
for i in $(seq ${REPS:-2}); do
  for lib in ${LIBS:-libcgck_base.so libcgck.so}; do
    echo "$lib" >> gpurun_out/ab_lib.log
    CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/$lib timeout -k 10 150 python tools/sweep.py ${SWEEP_ARGS:---variants slot2 --workloads imix --rounds 3} 2>/dev/null | grep median >> gpurun_out/ab_lib.log || exit 1
    if [ -n "$RSS" ]; then
      CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/$lib timeout -k 10 60 python tools/rss_bench.py --reps 20 2>/dev/null | grep '"hash"' >> gpurun_out/ab_lib.log || exit 1
    fi
  done
done
echo done
