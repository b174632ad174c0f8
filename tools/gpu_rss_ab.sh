#!/bin/bash
# In-process A/B of the Toeplitz batch kernel: the product's byte tables
# (libcgck_lab.so default, toeplitz12x4_ab_kernel<12>) against 12-bit-table
# variants built by tools/build_variant.sh (t12_d<depth>_<threads>.so).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rss_ab}
mkdir -p $O
for v in t12_d4_1024 t12_d3_1024 t12_d8_512 t12_d12_256; do
	[ -f con-gen_amd/$v.so ] || continue
	timeout -k 10 150 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck_lab.so,con-gen_amd/$v.so \
		--workloads rss --rounds 5 > $O/$v.log 2>&1
	rc=$?
	echo "$v rc=$rc"; tail -2 $O/$v.log | head -1
	[ $rc -eq 0 ] || exit $rc
done
