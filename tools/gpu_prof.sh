# rocprofv3 passes over bench.py (kernel trace + stats, then one PMC counter
# per pass, as MI355X_MICROARCH.md's HBM section prescribes).  Outputs under
# gpurun_out/prof_*; copy the summaries to profiles/ afterwards.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out
ARGS=${BENCH_ARGS:---steps 10 --warmup 3 --no-cpu --no-pmc}
timeout -k 10 120 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_trace -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_trace.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/prof_write.log 2>&1
echo "exit=$?"
