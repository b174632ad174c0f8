cd $GRAFT_REPO_ROOT
O=gpurun_out/rss_store; mkdir -p $O
for v in rss_plain rss_sc1 rss_d8; do
	timeout -k 10 200 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck_lab.so,con-gen_amd/$v.so --workloads rss --rounds 4 --launches 30 > $O/$v.log 2>&1 || exit 1
	echo "$v"; grep "rss:" $O/$v.log
done
