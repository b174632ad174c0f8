# A/B of two library builds on the burst server's latency, interleaved in
# one GPU call: tools/ab_head and tools/ab_new hold libcgck.so /
# libcgck_lab.so of each (tools/build_variant.sh); srvlat and txloop's lone
# and coalesced rows run against each in turn (LD_LIBRARY_PATH).
#   bash tools/ab_server.sh OUTDIR
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
for i in 1 2; do
	for v in head new; do
		LD_LIBRARY_PATH=$PWD/tools/ab_$v timeout -k 10 120 tools/srvlat 64 > $O/srvlat_${v}_$i.log 2>&1 || exit 1
		LD_LIBRARY_PATH=$PWD/tools/ab_$v timeout -k 10 120 tools/srvlat 64 fill > $O/srvlat_fill_${v}_$i.log 2>&1 || exit 1
		LD_LIBRARY_PATH=$PWD/tools/ab_$v TXLOOP_BURSTS=1,16,64,256,2048 TXLOOP_NS=250 timeout -k 10 200 tools/txloop 0.1 > $O/txloop_${v}_$i.log 2>&1 || exit 1
		echo "$v $i done"
	done
done
