# lpa pipeline depth A/B on one box: parity of the 3- and 4-deep variants through the
# forced-family test, then 64 B rates for depth 2/3/4 x blocks per CU
# (DEPTHS / CELLS override: CELLS is a comma list of env settings).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/lpa_depth.log
for d in ${DEPTHS:-3 4}; do CGCK_LPA_DEPTH=$d timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "family" -m gpu >> gpurun_out/lpa_depth.log 2>&1 || exit 1; done
run() { echo "$1" >> gpurun_out/lpa_depth.log; env $1 timeout -k 10 120 python tools/sweep.py --variants auto --workloads 64 --rounds 3 2>/dev/null | grep "64 " >> gpurun_out/lpa_depth.log || exit 1; }
if [ -n "$CELLS" ]; then IFS=, read -ra cells <<< "$CELLS"; else
cells=("CGCK_LPA_DEPTH=2 CGCK_LPA_BPC=3" "CGCK_LPA_DEPTH=3 CGCK_LPA_BPC=1" "CGCK_LPA_DEPTH=3 CGCK_LPA_BPC=2"
       "CGCK_LPA_DEPTH=4 CGCK_LPA_BPC=1" "CGCK_LPA_DEPTH=4 CGCK_LPA_BPC=2" "CGCK_LPA_DEPTH=2 CGCK_LPA_BPC=3"
       "CGCK_LPA_DEPTH=3 CGCK_LPA_BPC=1" "CGCK_LPA_DEPTH=4 CGCK_LPA_BPC=1"); fi
for c in "${cells[@]}"; do
  run "$c"
done
echo done
