# Round 4: the registered-ring server diagnostic (round-3 library, then this
# tree's), then the whole GPU suite.  Stops at the first abnormal exit.
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTDIR:-r4a}
mkdir -p $O
run() { # name seconds cmd...
	local name=$1 secs=$2; shift 2
	timeout -k 10 $secs "$@" > $O/$name.log 2>&1
	local rc=$?
	echo "$name rc=$rc"; tail -2 $O/$name.log
	return $rc
}
run stress_r3 110 python -u tools/reg_stress.py 60 plain tools/r3lib/libcgck.so
rc=$?; [ $rc -le 1 ] || exit $rc
run stress_new 110 python -u tools/reg_stress.py 60 plain
rc=$?; [ $rc -le 1 ] || exit $rc
run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
