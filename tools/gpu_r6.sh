# Round 6 GPU steps: bash tools/gpu_r6.sh OUTDIR step [step ...]
#   tests   — the whole -m gpu suite (slow ones included)
#   quick   — the burst / window tests only
#   txburst — tools/txburst 0.2 (all burst rows, pipelined included)
#   bench   — python bench.py (default N=1 line)
#   stress  — tools/reg_stress.py 60 plain
# Each step has its own time limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
shift
mkdir -p $O
rocminfo 2>/dev/null | grep -m2 -E "Marketing" > $O/info.txt || true
run() { # name seconds cmd...
	local name=$1 secs=$2; shift 2
	timeout -k 10 $secs "$@" > $O/$name.log 2>&1
	local rc=$?
	echo "$name rc=$rc"; tail -3 $O/$name.log
	return $rc
}
for step in "$@"; do
	case $step in
	tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread || exit 1 ;;
	cycles) for i in 1 2 3; do run pytest_cycles$i 300 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -k "not reregister or reregister" || true; done ;;
	testsk) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread || true ;;
	lab) # workgroups but the leader start their slices 20 us late (opts 512), so a
		# stale done word taken for served shows as outputs not yet written
		CGCK_SERVER_OPTS=512 run pytest_lab 300 python -u -m pytest tests/test_gpu_burst_lab.py -m "gpu and lab" -x -v --timeout 120 --timeout-method thread || exit 1
		# the control: the same test with the done-word refresh switched off must fail
		CGCK_SERVER_OPTS=528 run pytest_lab_norefresh 300 python -u -m pytest tests/test_gpu_burst_lab.py -m "gpu and lab" -v --timeout 120 --timeout-method thread
		echo "control (refresh off) rc=$?" ;;
	srvlatab) # lab: the read phase without the system-scope acquire (32) or with an agent-scope one (64)
		run srvlat_64_base 120 tools/srvlat 64 || exit 1
		CGCK_SERVER_OPTS=64 run srvlat_64_agentacq 120 tools/srvlat 64
		CGCK_SERVER_OPTS=128 run srvlat_64_l1inv 120 tools/srvlat 64 ;;
	srvlatrel) # the publish after the stores' own completion against the system release (opts 2048)
		for i in 1 2; do
			run srvlat_64_new$i 120 tools/srvlat 64 || exit 1
			run srvlat_64_fill_new$i 120 tools/srvlat 64 fill || exit 1
			CGCK_SERVER_OPTS=2048 run srvlat_64_rel$i 120 tools/srvlat 64 || exit 1
			CGCK_SERVER_OPTS=2048 run srvlat_64_fill_rel$i 120 tools/srvlat 64 fill || exit 1
		done ;;
	srvlatlds) # a small request's block in LDS against the scratch copy (opts 4096)
		for i in 1 2; do
			run srvlat_64_lds$i 120 tools/srvlat 64 || exit 1
			run srvlat_64_fill_lds$i 120 tools/srvlat 64 fill || exit 1
			CGCK_SERVER_OPTS=4096 run srvlat_64_scr$i 120 tools/srvlat 64 || exit 1
			CGCK_SERVER_OPTS=4096 run srvlat_64_fill_scr$i 120 tools/srvlat 64 fill || exit 1
		done ;;
	srvlat) run srvlat_64 120 tools/srvlat 64 || exit 1
		run srvlat_64_raw 120 tools/srvlat 64 raw || exit 1 ;;
	quick) run pytest_quick 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "burst or window or pipelined or rx_post or tx_" || exit 1 ;;
	txburst) run txburst 400 tools/txburst 0.2 || exit 1 ;;
	txloop) # pinned to the middle CPU of the allowed set, as bench.py pins it
		C=$(python3 -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[len(c)//2])")
		run txloop 400 taskset -c $C tools/txloop 0.2 || exit 1 ;;
	split) TXLOOP_SPLIT=1 run txloop_split 60 tools/txloop 0.5 || exit 1
		TXLOOP_SPLIT=2 run txloop_split_reply 60 tools/txloop 0.5 || exit 1 ;;
	splitlab) # the split timing with the Poster's phases (lab library)
		for r in 1 16 64 256; do
			TXLOOP_SPLIT=1 TXLOOP_SPLIT_R=$r run txloop_lab_split1_r$r 60 tools/txloop_lab 0.5 || exit 1
		done
		TXLOOP_SPLIT=2 TXLOOP_SPLIT_R=64 run txloop_lab_split2_r64 60 tools/txloop_lab 0.5 || exit 1 ;;
	splitn) # the split timing per burst size (250 ns a frame), RX only and with replies
		for r in 4 16 64 256; do
			for m in 1 2; do
				TXLOOP_SPLIT=$m TXLOOP_SPLIT_R=$r run txloop_split${m}_r$r 60 tools/txloop 0.5 || exit 1
			done
		done ;;
	e2e) run e2e 300 python -u tools/e2e.py || exit 1 ;;
	lpdab) # lab lpd variants against the product kernel, one process each (64 B)
		for cfg in "64 6 2" "64 5 2" "32 8 5" "64 6 5" "16 8 2"; do
			set -- $cfg
			CGCK_LPD_C=$1 CGCK_LPD_WPC=$2 CGCK_LPD_SP=$3 run lpdab_c$1_w$2_sp$3 120 python -u tools/ab_inproc.py \
				--libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_lab.so --workloads 64 --rounds 5 || exit 1
		done ;;
	rss) run rss_steady 200 python -u tools/rss_steady.py || exit 1 ;;
	txloop128) TXLOOP_LEN=128 run txloop128 400 tools/txloop 0.2 || exit 1 ;;
	txlens) # con-gen's typical frames (54-130 B): 128 B beside 64 B
		TXBURST_LENS=128,64 run txburst_128 400 tools/txburst 0.2 || exit 1 ;;
	txstack) # the same rows with 150 us of other stack work between bursts
		TXBURST_STACK_US=150 run txburst_stack150 400 tools/txburst 0.2 || exit 1 ;;
	txkstore) # lab: the kernel stores the posted fills' fields (CGCK_STORE) instead of the host
		LD_LIBRARY_PATH=$PWD/tools/labso CGCK_TX_KSTORE=1 run txburst_kstore 400 tools/txburst 0.2 || exit 1 ;;
	txtouch) # the TX rows with each frame's line written by the core before the clock starts
		TXBURST_PRETOUCH=1 run txburst_pretouch 400 tools/txburst 0.2 || exit 1 ;;
	bench) run bench 600 python -u bench.py || exit 1 ;;
	smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1 ;;
	bench2) run bench_n2 600 python -u bench.py --gpus 2 --allow-shared-devices --steps 5 --warmup 2 --no-burst || exit 1 ;;
	stress) # mmap'd rings: numpy's own allocations can come from the brk heap,
		# which cgck_host_register refuses
		run stress 110 python -u tools/reg_stress.py 60 mmap || exit 1 ;;
	stressm) for m in heap plain lock mmap; do run stress_$m 110 python -u tools/reg_stress.py 40 $m || exit 1; done ;;
	stress3) run stress_r3 110 python -u tools/reg_stress.py 30 plain tools/r3lib/libcgck.so || exit 1
		run stress_new 110 python -u tools/reg_stress.py 30 plain || exit 1 ;;
	lpwab) # lpw on each IMIX layout, full kernel vs its DMA rounds alone (lab build)
		for w in imixp imix ring; do
			for k in 1 2; do
				CGCK_LIB=con-gen_amd/libcgck_lab.so run lpw_${w}_full$k 120 python -u tools/one_workload.py $w --launches 10 || exit 1
				CGCK_LIB=con-gen_amd/libcgck_lab.so CGCK_LPW_NOCONS=1 run lpw_${w}_rounds$k 120 python -u tools/one_workload.py $w --launches 10 || exit 1
			done
		done ;;
	steady) run steady 300 python -u tools/steady.py --launches 120 --repeat 2 || exit 1 ;;
	workers) # N worker threads, each with its own ring, context and burst server
		run workers_q4 600 tools/txloop 0.3 || exit 1 ;;
	workersq) # the same with more hardware queues per process (each resident server needs its own)
		GPU_MAX_HW_QUEUES=32 run workers_q32 600 tools/txloop 0.3 || exit 1 ;;
	workersk) # the knee: 16..32 workers, the stack work spun, then slept (the CPU-quota control)
		TXLOOP_WORKERS=16,20,24,28,32 run workers_knee 600 tools/txloop 0.3 || exit 1
		TXLOOP_SLEEP=1 TXLOOP_WORKERS=1,16,24,32 run workers_sleep 600 tools/txloop 0.3 || exit 1 ;;
	txfull) # the full-transmit-ring regime: replies built in the stack-local packet (computed synchronously)
		C=$(python3 -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[len(c)//2])")
		TXLOOP_MIXES=1,2,3 TXLOOP_BURSTS=1,16,64,256 run txloop_full 300 taskset -c $C tools/txloop 0.2 || exit 1 ;;
	doorab) # the device-memory doorbell and small-block slots against the host-memory mailbox (lab build)
		for i in 1 2; do
			run srvlat_64_vram$i 120 tools/srvlat 64 || exit 1
			CGCK_BURST_HOST_DOOR=1 run srvlat_64_host$i 120 tools/srvlat 64 || exit 1
			run srvlat_64_fill_vram$i 120 tools/srvlat 64 fill || exit 1
			CGCK_BURST_HOST_DOOR=1 run srvlat_64_fill_host$i 120 tools/srvlat 64 fill || exit 1
		done ;;
	doorab2) # the doorbell A/B after the stop word moved beside it: host mailbox and blocks (HOST_DOOR),
		# doorbell and small blocks in device memory (default), doorbell alone (VRAM_MAX=0); srvlat and the
		# loop's small bursts, interleaved, twice
		for i in 1 2; do
			for m in host vram door; do
				case $m in host) E="CGCK_BURST_HOST_DOOR=1";; vram) E="X=1";; door) E="CGCK_BURST_VRAM_MAX=0";; esac
				env $E timeout -k 10 120 tools/srvlat 64 > $O/srvlat_64_${m}$i.log 2>&1 || exit 1
				env $E timeout -k 10 120 tools/srvlat 64 fill > $O/srvlat_64_fill_${m}$i.log 2>&1 || exit 1
				env $E TXLOOP_BURSTS=1,16,64,256 TXLOOP_NS=250 TXLOOP_MIXES=0,1 timeout -k 10 200 tools/txloop_lab 0.15 > $O/txloop_${m}$i.log 2>&1 || exit 1
				echo "$m $i"; head -1 $O/srvlat_64_${m}$i.log
			done
		done ;;
	doorab3) # pinned, interleaved: the host mailbox (HOST_DOOR) against the default (doorbell in device
		# memory; synchronous requests' small blocks there too, posted ones' in host staging)
		C=$(python3 -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[len(c)//2])")
		for i in 1 2 3; do
			for m in host dflt; do
				case $m in host) E="CGCK_BURST_HOST_DOOR=1";; dflt) E="X=1";; esac
				env $E timeout -k 10 120 taskset -c $C tools/srvlat 64 > $O/srvlat_64_${m}$i.log 2>&1 || exit 1
				env $E TXLOOP_BURSTS=1,16,64,256 TXLOOP_NS=250 TXLOOP_MIXES=0,1 timeout -k 10 200 taskset -c $C tools/txloop_lab 0.15 > $O/txloop_${m}$i.log 2>&1 || exit 1
				echo "$m $i"; head -1 $O/srvlat_64_${m}$i.log
			done
		done ;;
	smallonly) # the staged small path in a server kernel without the other paths (lab -DCGCK_SERVER_SMALL_ONLY=1,
		# con-gen_amd/small/libcgck_lab.so) against the full lab server; bursts past 64 are refused there (srvlat stops)
		for i in 1 2; do for m in full small; do for k in verify raw; do
			D=con-gen_amd; [ $m = small ] && D=con-gen_amd/small
			LD_LIBRARY_PATH=$D timeout -k 10 120 taskset -c 2 tools/srvlat 64 $k > $O/srvlat_64_${k}_$m$i.log 2>&1 || true
			echo "$k $m $i $(head -1 $O/srvlat_64_${k}_$m$i.log)"
		done; done; done ;;
	bodylive) # the body alone with 20 uniform 64-bit values live across it, against without
		for m in raw verify; do for sp in spec live spec live; do
			timeout -k 10 60 tools/bodylat 1 64 $m 2000 $sp >> $O/bodylive.log 2>&1 || exit 1
		done; done
		cat $O/bodylive.log ;;
	bodysplit) # the one-workgroup body inside the server (srvlat body_cycles) against the same body alone (bodylat)
		for k in verify fill raw; do
			timeout -k 10 120 taskset -c 2 tools/srvlat 64 $k > $O/srvlat_64_$k.log 2>&1 || exit 1
			echo "$k $(head -1 $O/srvlat_64_$k.log)"
		done
		for k in verify raw; do
			CGCK_SERVER_OPTS=16384 timeout -k 10 120 taskset -c 2 tools/srvlat 64 $k > $O/srvlat_64_${k}_twice.log 2>&1 || exit 1
			echo "$k twice $(head -1 $O/srvlat_64_${k}_twice.log)"
		done
		for m in raw verify fill; do timeout -k 10 60 tools/bodylat 1 64 $m 2000 spec >> $O/bodylat.log 2>&1 || exit 1; done
		cat $O/bodylat.log ;;
	specloop) # pinned, interleaved: the windows with the body compiled per flag set against the run-time flags (lab opts 8192)
		C=$(python3 -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[len(c)//2])")
		for i in 1 2 3; do
			for m in spec rt; do
				case $m in rt) E="CGCK_SERVER_OPTS=8192";; spec) E="CGCK_SERVER_OPTS=0";; esac
				env $E TXLOOP_BURSTS=1,16,64,256 TXLOOP_NS=250 TXLOOP_MIXES=0,1 timeout -k 10 200 taskset -c $C tools/txloop_lab 0.15 > $O/txloop_${m}$i.log 2>&1 || exit 1
				echo "$m $i"
			done
		done ;;
	stall) # repro of the 200 ms loop stall (rx+reply, 0 ns, 256 frames, coalesced after sync), lab then product
		C=$(python3 -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[len(c)//2])")
		TXLOOP_MIXES=1 TXLOOP_NS=0 TXLOOP_BURSTS=64,256 TXLOOP_REPEAT=12 timeout -k 10 280 taskset -c $C tools/txloop_lab 0.1 > $O/stall_lab.log 2> $O/stall_lab.err || exit 1
		TXLOOP_MIXES=1 TXLOOP_NS=0 TXLOOP_BURSTS=64,256 TXLOOP_REPEAT=12 timeout -k 10 280 taskset -c $C tools/txloop 0.1 > $O/stall.log 2> $O/stall.err || exit 1
		grep -c slow $O/stall_lab.err $O/stall.err || true ;;
	lpwpmc) # where lpw's time goes: SQ counters per workload (one pass of 8 SQ counters each), and the
		# lab's DMA-rounds-only variant beside the full kernel
		cd /tmp && export TMPDIR=/tmp
		P="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
		for w in imixp ring 1500; do
			timeout -s KILL 120 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/pmc_$w -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/one_workload.py $w --launches 3 > $GRAFT_REPO_ROOT/$O/pmc_$w.log 2>&1 || exit 1
		done
		for w in imixp ring; do
			CGCK_LIB=$GRAFT_REPO_ROOT/con-gen_amd/libcgck_lab.so CGCK_LPW_NOCONS=1 timeout -s KILL 120 rocprofv3 --pmc $P -d $GRAFT_REPO_ROOT/$O/pmc_${w}_dma -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/one_workload.py $w --launches 3 > $GRAFT_REPO_ROOT/$O/pmc_${w}_dma.log 2>&1 || exit 1
		done
		cd $GRAFT_REPO_ROOT ;;
	postedab) # lab: posted requests' small blocks (up to 512 B: ~37 descriptors) in device memory too, against
		# the product's choice (host staging), pinned and interleaved: the lone burst and the worker's cost
		C=$(python3 -c "import os; c=sorted(os.sched_getaffinity(0)); print(c[len(c)//2])")
		for i in 1 2 3; do
			for m in host vram; do
				case $m in host) E="X=1";; vram) E="CGCK_BURST_VRAM_POSTED_MAX=512";; esac
				env $E TXLOOP_BURSTS=1,4,16,32 TXLOOP_NS=250 TXLOOP_MIXES=0,1 timeout -k 10 200 taskset -c $C tools/txloop_lab 0.15 > $O/txloop_posted_${m}$i.log 2>&1 || exit 1
			done
		done ;;
	lpwab2) # in-process A/B of lpw (libcgck_base.so: the previous build) on the IMIX layouts, twice
		for i in 1 2; do
			run lpwab$i 300 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck_base.so,con-gen_amd/libcgck.so --workloads imixp,ring,imix --rounds 6 || exit 1
		done ;;
	lpwdma) # lab variants: smaller lpw windows (6 / 4 KiB) with more waves per CU, in-process against the product
		CGCK_LPW_WPC=10 run lpwdma6 300 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_v6.so --workloads imixp,ring --rounds 6 || exit 1
		CGCK_LPW_WPC=12 run lpwdma4 300 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_v4.so --workloads imixp,ring --rounds 6 || exit 1
		CGCK_LPW_WPC=8 run lpwdma6w8 300 python -u tools/ab_inproc.py --libs con-gen_amd/libcgck.so,con-gen_amd/libcgck_v6.so --workloads imixp,ring --rounds 6 || exit 1 ;;
	spec) # the one-workgroup body compiled per flag set: srvlat (verify staged / fill in place), pinned
		# against the run-time flags (lab opts 8192), interleaved on the same CPU
		for i in 1 2 3; do for m in spec rt; do
			E=CGCK_SERVER_OPTS=0; [ $m = rt ] && E=CGCK_SERVER_OPTS=8192
			for k in verify fill raw; do
				env $E timeout -k 10 120 taskset -c 2 tools/srvlat 64 $k > $O/srvlat_64_${k}_$m$i.log 2>&1 || exit 1
				echo "$k $m $i $(head -1 $O/srvlat_64_${k}_$m$i.log)"
			done
		done; done ;;
	bodylat) # the server body's cycles for one small request, by mode and burst (tools/bodylat.hip)
		for sp in rt spec; do
			for m in raw verify fill; do for n in 1 64; do
				timeout -k 10 60 tools/bodylat $n 64 $m 2000 $sp >> $O/bodylat.log 2>&1 || exit 1
			done; done
			timeout -k 10 60 tools/bodylat 1 1500 verify 2000 $sp >> $O/bodylat.log 2>&1 || exit 1
		done
		cat $O/bodylat.log ;;
	lpwtests) run pytest_lpw 300 python -u -m pytest tests/test_gpu_lpw.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1 ;;
	workers4) TXLOOP_WORKERS=1,8,12,16,32 run workers 600 tools/txloop 0.3 || exit 1 ;;
	vramdb) run vramdb 120 tools/vramdb 0.3 || exit 1 ;;
	shards) run shards 600 python -u -m pytest tests/test_gpu_shards.py -m gpu -x -v -s --timeout 500 --timeout-method thread || exit 1 ;;
	profbench) BENCH_ARGS="--steps 10 --warmup 3 --no-cpu --no-pmc --no-burst" bash tools/gpu_prof.sh || exit 1 ;;
	prof) bash tools/gpu_prof_layouts.sh $(basename $O)/prof || exit 1 ;;
	*) echo "unknown step $step"; exit 2 ;;
	esac
done
