# A/B of two library builds on the poll loop's host cost, interleaved in one
# GPU call: tools/ab_head and tools/ab_new (libcgck.so of each,
# tools/build_variant.sh); txloop's split timing and coalesced rows.
#   bash tools/ab_loop.sh OUTDIR
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
# $2: a core to pin every run to (taskset), so both builds run on the same one
PIN=${2:+taskset -c $2}
for i in 1 2 3; do
	for v in head new; do
		for m in 1 2; do
			for r in 1 16 32; do
				LD_LIBRARY_PATH=$PWD/tools/ab_$v TXLOOP_SPLIT=$m TXLOOP_SPLIT_R=$r timeout -k 10 60 $PIN tools/txloop 0.25 > $O/split${m}_r${r}_${v}_$i.log 2>&1 || exit 1
			done
		done
		LD_LIBRARY_PATH=$PWD/tools/ab_$v TXLOOP_BURSTS=1,4,16,32,64 TXLOOP_NS=250 timeout -k 10 200 $PIN tools/txloop 0.1 > $O/txloop_${v}_$i.log 2>&1 || exit 1
		echo "$v $i done"
	done
done
