# Burst-path iteration on the GPU box: the server / window parity tests, then
# the C-ABI burst harness (tools/txburst) and the reference CPU loop over the
# same bursts.  Every GPU step has its own limit; the first failure ends the
# call.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_windows.py tests/test_gpu_parity.py -k "burst or window" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_burst.log 2>&1 && echo "burst tests ok" && \
timeout -k 10 300 ./tools/txburst 0.15 > gpurun_out/txburst.log 2> gpurun_out/txburst.err && echo "txburst ok" && \
timeout -k 10 200 python -c "
import json, bench
print(json.dumps(bench.cpu_burst()))" > gpurun_out/cpu_burst.json 2>&1 && echo "cpu ok"
echo "exit=$?"
