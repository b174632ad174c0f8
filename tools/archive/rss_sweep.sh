# A/B timing of the batched Toeplitz hash (tools/rss_bench.py) under the
# CGCK_RSS_VAR / CGCK_RSS_BPC / CGCK_RSS_DEPTH knobs (cells var:bpc[:depth];
# CGCK_DST_ITERS / CGCK_DST_WGS for the dst-cache build).  DEPTHS: ring depths
# whose parity is checked first (tests/test_gpu_rss.py).  GPU box only; each
# cell its own process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/rsweep.log
for d in ${DEPTHS:-}; do
  CGCK_RSS_DEPTH=$d timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_rss.py -m gpu >> gpurun_out/rsweep.log 2>&1 || exit 1
done
for cell in ${CELLS:-0:8 2:8 2:4 2:16 1:8 0:8 2:8}; do
  echo "var:bpc:depth=$cell" >> gpurun_out/rsweep.log
  IFS=: read -r v b d <<< "$cell"
  CGCK_RSS_VAR=$v CGCK_RSS_BPC=$b CGCK_RSS_DEPTH=${d:-2} timeout -k 10 60 python tools/rss_bench.py --reps 20 2>/dev/null | grep '"hash"' >> gpurun_out/rsweep.log || exit 1
done
echo done
