# 64 B alone (bench.py --only 64): contiguous (CGCK_DEV_ALLOC_FLAGS=4) vs plain hipMalloc (default)
# inputs, alternating processes on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
	for f in contig plain; do
		if [ $f = contig ]; then export CGCK_DEV_ALLOC_FLAGS=4; else unset CGCK_DEV_ALLOC_FLAGS; fi
		CGCK_ALLOC_VERBOSE=1 timeout -k 10 120 python -u bench.py --only 64 --no-cpu --no-burst --no-rss --steps 10 --warmup 3 > gpurun_out/alloc64_$f$i.log 2>&1 || { echo "$f$i failed"; tail -n 5 gpurun_out/alloc64_$f$i.log; exit 1; }
		tail -n 1 gpurun_out/alloc64_$f$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('$f$i', '64 %.3f' % e['64B']['hbm_frac'])"
	done
done
echo "exit=0"
