set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/info.txt || true
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m "gpu and not slow" -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_slow.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
echo "exit=$?"
