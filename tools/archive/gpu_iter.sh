# Iteration run on the GPU box: parity under every kernel family listed in
# $FAMS, the full-size tests, then the in-process A/B sweep.  Every GPU step
# has its own time limit; steps are chained with && so the first failure
# ends the call.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ok=0
for f in ${FAMS:-group lpp}; do
  CGCK_KERNEL=$f timeout -k 10 300 python -m pytest tests -m "gpu and not slow" -x -q > gpurun_out/pytest_$f.log 2>&1 || { ok=1; echo "parity failed under $f"; break; }
done
[ $ok = 0 ] && \
timeout -k 10 300 python -m pytest tests -m "gpu and slow" -x -q > gpurun_out/pytest_slow.log 2>&1 && \
timeout -k 10 400 python tools/sweep.py ${SWEEP_ARGS:-} > gpurun_out/sweep.log 2>&1 && \
{ [ -z "${SWEEP2_ARGS:-}" ] || timeout -k 10 400 python tools/sweep.py $SWEEP2_ARGS > gpurun_out/sweep2.log 2>&1; }
echo "exit=$?"
