# Diagnostics: read-probe variants x sizes, then SQ / TA / TCP counter passes
# over bench.py (one counter group per pass, no tracing domains).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && PROBE_MB=${PROBE_MB:-1024,24000} PROBE_VARIANTS=${PROBE_VARIANTS:-0,4,6,7,8} timeout -k 10 300 python tools/probe.py > gpurun_out/probe.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu}
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp -d $R/gpurun_out/diag_$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/diag_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "exit=0"
