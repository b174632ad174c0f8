# Counter passes over bench.py (no tracing domains; one group per pass; each
# pass under its own short time limit).  Groups come from $PMC_PGRPS
# (';'-separated).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 3 --warmup 1 --no-cpu}
IFS=';' read -ra PGRPS <<< "${PMC_PGRPS:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY}"
i=0
for grp in "${PGRPS[@]}"; do
  i=$((i+1))
  echo "pass $i: $grp" >> $R/gpurun_out/pmc_progress.txt
  timeout -k 10 240 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc_$i -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_$i.log 2>&1 || { echo "pass $i failed" >> $R/gpurun_out/pmc_progress.txt; exit 1; }
done
echo "exit=0"
