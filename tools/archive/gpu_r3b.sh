# Round-3 check + the lpw A/Bs: the round check (tools/gpu_r3.sh), slot2 vs
# lpw per layout (tools/family_ab.py), then the writer-wave lpw (lab build,
# CGCK_LPW_W=1) against the product lpw in one process (tools/ab_inproc.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_r3.sh | tee gpurun_out/r3.out | tail -1 | grep -q "exit=0" || { echo "round check failed"; cat gpurun_out/r3.out; exit 1; }
echo "round check ok"
timeout -k 10 300 python tools/family_ab.py --families slot2,lpw --layouts packed,ring,sring > gpurun_out/family_ab2.log 2>&1 && echo "family ab ok" && \
CGCK_LPW_W=1 timeout -k 10 300 python tools/ab_inproc.py --libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_lab.so --workloads imix,ring --rounds 5 > gpurun_out/ab_lpw_writer.log 2>&1 && echo "writer ab ok"
echo "exit=$?"
