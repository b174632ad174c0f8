# In-process A/B of the 1500 B kernel: the lab build against a variant
# (tools/build_variant.sh), alternating launch blocks on one buffer; outputs
# compared byte for byte.
cd $GRAFT_REPO_ROOT
O=gpurun_out/dstr_ab; mkdir -p $O
for v in "$@"; do
	timeout -k 10 300 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck_lab.so,con-gen_amd/$v.so --workloads 1500 --rounds 8 > $O/$v.log 2>&1 || exit 1
	echo "$v"; grep "1500:" $O/$v.log
done
