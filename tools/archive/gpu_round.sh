# Round evidence in one GPU call: smoke + parity + bench (gpu_check.sh), the
# rocprofv3 trace/stats and FETCH/WRITE passes (gpu_prof.sh), then the
# end-to-end pinned-host rates (tools/e2e.py).  Stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
bash tools/gpu_check.sh > gpurun_out/check.out 2>&1; grep -q "exit=0" gpurun_out/check.out || { echo "check failed"; cat gpurun_out/check.out; exit 1; }
echo "check ok"; tail -n 1 gpurun_out/bench.log
bash tools/gpu_prof.sh > gpurun_out/prof.out 2>&1; grep -q "exit=0" gpurun_out/prof.out || { echo "prof failed"; cat gpurun_out/prof.out; exit 1; }
echo "prof ok"
cd $R && timeout -k 10 300 python tools/e2e.py > gpurun_out/e2e.log 2>&1 || { echo "e2e failed"; tail -n 20 gpurun_out/e2e.log; exit 1; }
tail -n 3 gpurun_out/e2e.log
echo "exit=0"
