# Contiguous (default) vs plain hipMalloc device allocations, alternating
# bench.py processes on one box (CGCK_DEV_ALLOC_FLAGS=4 selects contiguous).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
	for f in contig plain; do
		if [ $f = contig ]; then export CGCK_DEV_ALLOC_FLAGS=4; else unset CGCK_DEV_ALLOC_FLAGS; fi
		CGCK_ALLOC_VERBOSE=1 timeout -k 10 150 python -u bench.py --no-cpu --no-burst --steps 10 --warmup 3 > gpurun_out/alloc_$f$i.log 2>&1 || { echo "$f$i failed"; tail -n 5 gpurun_out/alloc_$f$i.log; exit 1; }
		grep -h "cgck_dev_alloc" gpurun_out/alloc_$f$i.log || true
		tail -n 1 gpurun_out/alloc_$f$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$f$i', '1500 %.3f' % d['roofline']['frac'], '64 %.3f' % e['64B']['hbm_frac'], 'imix %.3f' % e['imix']['hbm_frac'], 'rss %.3f' % e['rss_hash']['hbm_frac'])"
	done
done
echo "exit=0"
