# Blocks-per-CU sweep of the three checksum kernels on their BASELINE
# workloads (GPU box only; each cell its own process, knobs read once).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/bpc_sweep.log
run() { echo "$1" >> gpurun_out/bpc_sweep.log; env $1 timeout -k 10 120 python tools/sweep.py --variants auto --workloads $2 --rounds 3 2>/dev/null | grep "$2 " >> gpurun_out/bpc_sweep.log || exit 1; }
for b in ${GRP:-16 24 32 16}; do run "CGCK_GRP_BPC=$b" 1500; done
for b in ${LPA:-3 1 2 3}; do run "CGCK_LPA_BPC=$b" 64; done
for b in ${SLOT:-8 12 16 8}; do run "CGCK_BPC=$b" imix; done
echo done
