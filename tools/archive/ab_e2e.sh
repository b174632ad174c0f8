# e2e (tools/e2e.py) against product-build variants, interleaved in one GPU
# call: bash tools/ab_e2e.sh OUTDIR NAME... (con-gen_amd/NAME.so, through
# $CGCK_LIB; tools/build_variant.sh with VARIANT_PRODUCT=1 builds them).
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
shift
mkdir -p $O
for i in 1 2; do
	for v in "$@"; do
		CGCK_LIB=$PWD/con-gen_amd/$v.so timeout -k 10 300 python -u tools/e2e.py > $O/e2e_${v}_$i.log 2>&1 || exit 1
		echo "$v $i done"
	done
done
