# rocprofv3 per IMIX layout: one kernel-trace/stats pass
# and one FETCH_SIZE and one WRITE_SIZE pass over tools/one_workload.py for
# each of imixp (packed hint), imix (no hint) and ring (2048 B slots at +14),
# so each layout's lpw average and HBM bytes come from a kernel_stats.csv of
# their own.  Also 1500 and 64 for the same table.  Outputs: gpurun_out/$1/.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS:-imixp imix ring 1500 64}; do
	timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o run --output-format csv -- python3 $R/tools/one_workload.py $w --launches 10 > $O/trace_$w.log 2>&1 || exit 1
	timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$w -o run --output-format csv -- python3 $R/tools/one_workload.py $w --launches 3 > $O/fetch_$w.log 2>&1 || exit 1
	timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write_$w -o run --output-format csv -- python3 $R/tools/one_workload.py $w --launches 3 > $O/write_$w.log 2>&1 || exit 1
	echo "$w done"; cat $O/trace_$w.log | tail -1
done
