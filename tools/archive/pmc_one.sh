# PMC passes over tools/one_workload.py $WL (one kernel): HBM traffic, then
# the SQ instruction / wait mix.  Each pass under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
WL=${WL:-imixp}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/one_workload.py $WL > $R/gpurun_out/one_$WL.log 2>&1 || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc1_${WL}_$i -o run --output-format csv -- python3 $R/tools/one_workload.py $WL >> $R/gpurun_out/one_$WL.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "exit=0"
