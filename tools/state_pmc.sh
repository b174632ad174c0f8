# Counter passes over tools/state_pmc.py: TCC->EA read requests split by XCC,
# then by channel (TCC instance), then the average read latency and stalls;
# one rocprofv3 pass each under its own limit.  SKIP_SPLIT=1 runs only the last.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/state_pmc.py > $R/gpurun_out/state_plain.log 2>&1 || exit 1
[ -n "${SKIP_SPLIT:-}" ] || timeout -s KILL 90 rocprofv3 -E $R/tools/pmc/tcc_split.yaml --pmc RDREQ_XCC0 RDREQ_XCC1 RDREQ_XCC2 RDREQ_XCC3 RDREQ_XCC4 RDREQ_XCC5 RDREQ_XCC6 RDREQ_XCC7 -d $R/gpurun_out/pmc_xcc -o run --output-format csv -- python3 $R/tools/state_pmc.py > $R/gpurun_out/state_xcc.log 2>&1 || { echo "xcc pass failed"; tail -5 $R/gpurun_out/state_xcc.log; exit 1; }
[ -n "${SKIP_SPLIT:-}" ] || timeout -s KILL 90 rocprofv3 -E $R/tools/pmc/tcc_channels.yaml --pmc RDREQ_CH0 RDREQ_CH1 RDREQ_CH2 RDREQ_CH3 RDREQ_CH4 RDREQ_CH5 RDREQ_CH6 RDREQ_CH7 RDREQ_CH8 RDREQ_CH9 RDREQ_CH10 RDREQ_CH11 RDREQ_CH12 RDREQ_CH13 RDREQ_CH14 RDREQ_CH15 -d $R/gpurun_out/pmc_ch -o run --output-format csv -- python3 $R/tools/state_pmc.py > $R/gpurun_out/state_ch.log 2>&1 || { echo "channel pass failed"; tail -5 $R/gpurun_out/state_ch.log; exit 1; }
# average TCC->EA read latency (LEVEL / RDREQ) and DRAM-credit stalls per dispatch
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum -d $R/gpurun_out/pmc_lat -o run --output-format csv -- python3 $R/tools/state_pmc.py > $R/gpurun_out/state_lat.log 2>&1 || { echo "latency pass failed"; tail -5 $R/gpurun_out/state_lat.log; exit 1; }
echo "exit=0"
