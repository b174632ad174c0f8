# One GPU call: parity under $FAMS, A/B sweeps ($SWEEP_ARGS, $SWEEP2_ARGS),
# then the read probes ($PROBE_VARIANTS at $PROBE_MB).  Each step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_iter.sh > gpurun_out/iter.log 2>&1 || { echo "iter failed"; cat gpurun_out/iter.log; exit 1; }
grep -q "exit=0" gpurun_out/iter.log || { echo "iter failed"; cat gpurun_out/iter.log; exit 1; }
if [ -n "${PROBE_VARIANTS:-}" ]; then
  timeout -k 10 300 python tools/probe.py > gpurun_out/probe.log 2>&1 || { echo "probe failed"; exit 1; }
fi
echo "exit=0"
