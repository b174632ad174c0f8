# A/B timing of the Toeplitz RSS kernels (tools/rss_bench.py) under the
# CGCK_RSS_NIB / CGCK_DST_ITERS / CGCK_DST_WGS knobs.  GPU box only.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; : > gpurun_out/rsweep.log
for v in 0 1; do
  echo "nib=$v" >> gpurun_out/rsweep.log
  CGCK_RSS_NIB=$v timeout -k 10 60 python tools/rss_bench.py --reps 20 2>/dev/null | grep '"hash"' >> gpurun_out/rsweep.log || exit 1
done
echo done
