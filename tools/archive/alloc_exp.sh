# Server latency experiments (tools/txburst dropin): one in_cksum at a time
# through servers of the given (max_pkts[:max_bytes]) shapes, in order.
set -o pipefail
cd $GRAFT_REPO_ROOT
run() { echo "== $*"; timeout -k 10 60 ./tools/txburst 0.2 dropin "$@" || exit 1; }
{ run 0 64 256 1024 2048 0
} > gpurun_out/alloc_exp.log 2>&1
cat gpurun_out/alloc_exp.log
