# A/B timing of the batched Toeplitz hash (tools/rss_bench.py) under the
# CGCK_RSS_VAR / CGCK_RSS_BPC knobs (CGCK_DST_ITERS / CGCK_DST_WGS for the
# dst-cache build).  GPU box only; each cell its own process.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/rsweep.log
for cell in ${CELLS:-0:8 2:8 2:4 2:16 1:8 0:8 2:8}; do
  echo "var:bpc=$cell" >> gpurun_out/rsweep.log
  CGCK_RSS_VAR=${cell%%:*} CGCK_RSS_BPC=${cell##*:} timeout -k 10 60 python tools/rss_bench.py --reps 20 2>/dev/null | grep '"hash"' >> gpurun_out/rsweep.log || exit 1
done
echo done
