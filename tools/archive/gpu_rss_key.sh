# The RSS batch kernel under the bench's key and the sequential key, in one
# process (tools/ab_inproc.py, 30 launches per measurement), then the bench's
# own RSS leg, on one box.
cd $GRAFT_REPO_ROOT
O=gpurun_out/rss_key; mkdir -p $O
timeout -k 10 200 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_lab.so --workloads rss --rounds 4 --launches 30 > $O/ab_mskey.log 2>&1 || exit 1
AB_KEY=seq timeout -k 10 200 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_lab.so --workloads rss --rounds 4 --launches 30 > $O/ab_seqkey.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --only rss --no-cpu --no-pmc --no-burst > $O/bench.log 2>&1 || exit 1
grep "rss:" $O/ab_mskey.log $O/ab_seqkey.log
