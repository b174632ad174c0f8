#!/bin/sh
# Copy one round's GPU evidence from gpurun_out/ (merged back by gpurun after
# tools/gpu_r6.sh) into profiles/$ROUND/ (tracked).  Host side only.
set -eu
R=${1:-r01}
G=gpurun_out
D=profiles/$R
mkdir -p $D/rocprof
tail -n 1 $G/bench.log > $D/bench.json
for f in smoke.log pytest_gpu.log pytest_slow.log e2e.log info.txt; do
	[ -f $G/$f ] && cp $G/$f $D/$f
done
cp $G/prof_trace/run_kernel_stats.csv $D/rocprof/kernel_stats.csv
cp $G/prof_trace/run_kernel_trace.csv $D/rocprof/kernel_trace.csv
grep '^{"metric"' $G/prof_trace.log | tail -n 1 > $D/rocprof/bench_under_trace.json
cp $G/prof_fetch/run_counter_collection.csv $D/rocprof/pmc_fetch_size.csv
cp $G/prof_write/run_counter_collection.csv $D/rocprof/pmc_write_size.csv
python3 tools/pmc_traffic.py $G/prof_fetch $G/prof_write profiles/pmc_latest.json $D/rocprof/bench_under_trace.json > /dev/null
python3 tools/prof_check.py $D/rocprof/kernel_stats.csv $D/rocprof/bench_under_trace.json > $D/rocprof/kernel_vs_events.txt || true
echo "collected into $D"
