#!/usr/bin/env python3
"""Device-resident batched Internet-checksum benchmark (BASELINE.json metric).

One step = one pass of the hot path (IPv4 header checksum + TCP checksum with
pseudo-header, i.e. ip_cksum + tcp_cksum of subr.h:176-177, for every packet)
over one batch of synthetic packets already resident in HBM.  The headline
workload is BASELINE.json configs[2]: 16M x 1500 B packets on each GPU
(configs[4] = 128M x 1500 B over 8 GPUs, i.e. weak scaling at 16M per GPU).
The 64 B (configs[1]) and IMIX (configs[3]) batches are timed the same way and
reported as top-level value_64B / roofline_64B and value_imix / roofline_imix;
BASELINE configs[0] (1M x 64 B through the reference's CPU loop) is
cpu_baseline_cfg0.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Without a launcher, --gpus N > 1 starts torch.distributed.run with N ranks
as a child process (before anything touches the GPU) and relays rank 0's
line; under a launcher --gpus must equal WORLD_SIZE.
Rank 0 prints one JSON line.  One process per GPU: WORLD_SIZE above the
visible device count is refused unless --allow-shared-devices (rehearsals on
a one-GPU box).  The checker leg is the only part that touches oracle/: every
rank checks a sample of its own shard's outputs of this run against the
oracle referee (every 64 B packet, every 64th 1500 B / IMIX packet across
the whole shard; the totals are summed over ranks), and at N = 1 rank 0
times the reference's own subr.c checksum unit (oracle/_ref, when built) or
the oracle restatement on a bounded sample of the same workload as the CPU
baseline, and runs two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) per
device workload as child processes after the timed region, so roofline.traffic
is this box's HBM bytes per launch (--no-pmc: the committed summary).
Host-resident burst rates of SURVEY §8(f) ranks 1-2 (tools/txburst,
N = 1) are summarised under extra.burst; the full rows go to
gpurun_out/bench_burst.json.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "con-gen_amd"))

HBM_PEAK = 8.0e12          # MI355X HBM3E peak, B/s (MI355X_MICROARCH.md)
SEED = 0xC0C0              # splitmix64(seed = 0xC0C0 + shard)
METRIC = "Gpkts/s + GB/s device-resident checksum, 64B & 1500B batches; %HBM peak"


def shard_plan(rank, world, n_per_gpu):
    """Weak scaling, no collective on the data path: rank r owns packets
    [r*n, (r+1)*n) of the global batch, generated with seed 0xC0C0 + r."""
    return {"first": rank * n_per_gpu, "n": n_per_gpu, "seed": SEED + rank, "world": world}


def device_for(local_rank, world, ndev, allow_shared=False):
    """One process per GPU: local rank r drives device r.  More ranks than
    visible devices is refused (a line claiming N GPUs must run on N GPUs)
    unless a rehearsal asks for shared devices."""
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible (an MI355X is required)")
    if world > ndev and not allow_shared:
        raise SystemExit(f"bench.py: WORLD_SIZE {world} > {ndev} visible GPUs "
                         "(one rank per GPU; --allow-shared-devices for a rehearsal)")
    return local_rank % ndev


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (= ranks, one process each); without WORLD_SIZE in the environment "
                         "N > 1 starts torch.distributed.run with N ranks as a child process")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--packets", type=int, default=16 << 20, help="packets per GPU")
    ap.add_argument("--no-extra", action="store_true", help="skip the 64 B / IMIX lines")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-rss", action="store_true", help="skip the Toeplitz RSS lines")
    ap.add_argument("--no-burst", action="store_true", help="skip the host-resident burst lines")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the rocprofv3 --pmc traffic passes (roofline.traffic from profiles/ instead)")
    ap.add_argument("--only", choices=["1500", "64", "imix", "rss"], default=None,
                    help="time one workload only (profiling runs)")
    ap.add_argument("--allow-shared-devices", action="store_true",
                    help="let ranks share GPUs when WORLD_SIZE exceeds the visible devices "
                         "(rehearsals only: the line then says so)")
    return ap.parse_args(argv)


def launch_decision(gpus, env):
    """How this invocation runs (one process per GPU, as
    con-gen runs one worker per RSS queue, con-gen.c:1062-1100).
    Returns ("inprocess", world) or ("spawn", N).  Under a launcher
    (WORLD_SIZE set) --gpus must equal WORLD_SIZE; without one, --gpus N > 1
    asks this process to start the N ranks itself."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if gpus is None else gpus
        if n < 1:
            raise SystemExit(f"bench.py: --gpus {n} < 1")
        return ("spawn", n) if n > 1 else ("inprocess", 1)
    ws = int(ws)
    if gpus is not None and gpus != ws:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE {ws} "
                         "(one rank per GPU: launch with --nproc-per-node equal to --gpus)")
    return ("inprocess", ws)


def child_command(n, argv, port):
    """torch.distributed.run over N local ranks, rendezvous on 127.0.0.1,
    re-running this script with the same arguments (each rank then finds
    WORLD_SIZE = N and runs in-process)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """Run the N ranks as a child process (never exec: this process has not
    touched the GPU, and an exec after HIP init is forbidden on this pool).
    Rank 0's JSON line is relayed on stdout, everything else the child prints
    on stdout goes to stderr; the exit code is the child's."""
    import subprocess
    cmd = child_command(n, argv, free_port())
    print("bench.py: launching " + " ".join(cmd), file=sys.stderr, flush=True)
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = 0
    for line in p.stdout:
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
            lines += 1
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = p.wait()
    if rc == 0 and lines != 1:
        print(f"bench.py: the {n}-rank child printed {lines} result lines", file=sys.stderr)
        return 1
    return rc


class Dist:
    """Barrier and max-over-ranks; a no-op at world size 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, x):
        if self.world == 1:
            return x
        import torch
        t = torch.tensor([float(x)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def gather(self, obj):
        """Every rank's `obj`, in rank order (on every rank)."""
        if self.world == 1:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def timed(torch, dist, eng, cgck, step, steps, warmup):
    """W untimed steps, then K steps bracketed by barrier + synchronize on both
    sides.  Returns (max-over-ranks wall seconds, HIP-event ms per launch on
    the launch stream)."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    e0, e1 = cgck.Event(), cgck.Event()
    t0 = time.perf_counter()
    eng.record(e0)
    for _ in range(steps):
        step()
    eng.record(e1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    wall = dist.max(t1 - t0)
    return wall, cgck.Engine.elapsed_ms(e0, e1) / steps


def bench_strided(torch, dist, eng, cgck, n, size, plan, steps, warmup):
    buf = cgck.DeviceBuffer(n * size)
    out = cgck.DeviceBuffer(4 * n)
    eng.synth_strided(buf.ptr, n, size, size, plan["seed"])
    eng.sync()

    def step():
        eng.strided(buf.ptr, n, size, 0, size, cgck.GEN_BOTH, out.ptr)

    wall, ev_ms = timed(torch, dist, eng, cgck, step, steps, warmup)
    kernel = eng.last_kernel
    # every output of this run, downloaded once after the timed region, for the checker leg
    o = __import__("numpy").zeros(n, "uint32")
    out.download(o, stream=eng.stream)
    eng.sync()
    buf.free()
    out.free()
    return wall, ev_ms, o, kernel


def bench_imix(torch, dist, eng, cgck, n, plan, steps, warmup):
    """BASELINE configs[3]: the IMIX frames lie back to back in one buffer
    (cgck_synth_imix).  Timed with the caller's layout hint
    (cgck_set_desc_layout PACKED), then without it on the same buffer (the
    dispatcher's own choice: lpw detects the back-to-back steps itself), then
    the same frames in 2048 B receive-ring slots at +14; the same steps and
    warm-up each."""
    nbytes = cgck.load().cgck_imix_bytes(n)
    buf = cgck.DeviceBuffer(nbytes)
    desc = cgck.DeviceBuffer(12 * n)
    out = cgck.DeviceBuffer(4 * n)
    eng.synth_imix(buf.ptr, desc.ptr, n, plan["seed"])
    eng.set_desc_len_hint(nbytes // n)       # mean IMIX length (354 B)
    eng.sync()

    def step():
        eng.desc(buf.ptr, desc.ptr, n, cgck.GEN_BOTH, out.ptr)

    eng.set_desc_layout(cgck.LAYOUT_PACKED)
    wall, ev_ms = timed(torch, dist, eng, cgck, step, steps, warmup)
    kernel = eng.last_kernel
    o = __import__("numpy").zeros(n, "uint32")
    out.download(o, stream=eng.stream)
    eng.sync()
    eng.set_desc_layout(cgck.LAYOUT_ANY)
    wall_u, ev_u = timed(torch, dist, eng, cgck, step, steps, warmup)
    unhinted = {"kernel": eng.last_kernel, "kernel_ms": ev_u,
                "frac": (nbytes + 16 * n) / (ev_u * 1e-3) / HBM_PEAK}
    ou = __import__("numpy").zeros(n, "uint32")
    out.download(ou, stream=eng.stream)
    eng.sync()
    buf.free()
    desc.free()
    # The same IMIX frames in a receive ring: 2048 B slots, IPv4 at +14 (the
    # netmap layout, netmap.c:116-126), no layout hint.  Algorithmic bytes are
    # the frames', as for the packed set.
    rbuf = cgck.DeviceBuffer(n * RING_SLOT)
    rdesc = cgck.DeviceBuffer(12 * n)
    eng.synth_imix_ring(rbuf.ptr, rdesc.ptr, n, RING_SLOT, RING_L3, plan["seed"])
    eng.sync()
    wall_r, ev_r = timed(torch, dist, eng, cgck,
                         lambda: eng.desc(rbuf.ptr, rdesc.ptr, n, cgck.GEN_BOTH, out.ptr),
                         steps, warmup)
    ring = {"layout": f"{RING_SLOT} B slots, IPv4 at +{RING_L3}", "kernel": eng.last_kernel, "kernel_ms": ev_r,
            "frac": (nbytes + 16 * n) / (ev_r * 1e-3) / HBM_PEAK,
            "gpkt_s": n / (ev_r * 1e-3) / 1e9}
    orr = __import__("numpy").zeros(n, "uint32")
    out.download(orr, stream=eng.stream)
    eng.sync()
    eng.set_desc_len_hint(1500)
    rbuf.free()
    rdesc.free()
    out.free()
    return wall, ev_ms, nbytes, (o, ou, orr), kernel, unhinted, ring


RING_SLOT, RING_L3 = 2048, 14   # receive-ring layout of the IMIX frames (netmap slots)

RSS_KEY = bytes.fromhex("6d5a56da255b0ec24167253d43a38fb0d0ca2bcbae7b30b477cb2da38030f20c6a42b73bbeac01fa")
RSS_TUPLES = 64 << 20      # batched-hash tuples per GPU (805 MB: well past the 256 MB MALL)
RSS_DST = (4, 256, 8)      # dst-cache enumeration: laddrs x faddrs x 60536 ports, queues
RSS_WARMUP = 60            # launches before the hash leg's timed window (fresh buffers settle by ~40)


def bench_rss(torch, dist, eng, cgck, plan, steps, warmup):
    """SURVEY §8(f) rank 4.  (a) cgck_toeplitz over RSS_TUPLES dense 12-byte
    tuples in HBM (rss_hash4 layout, mask 0x7F): 16 algorithmic bytes per
    tuple.  (b) cgck_dst_cache over a full enumeration (no early cap):
    rank r builds the cache of RSS queue r % queues, as con-gen's thread r
    does (con-gen.c:337-342)."""
    import numpy as np
    n = RSS_TUPLES
    d = cgck.DeviceBuffer(n * 12 + 64)
    o = cgck.DeviceBuffer(4 * n)
    eng.synth_strided(d.ptr, (n * 12) // 1500, 1500, 1500, plan["seed"])
    eng.sync()
    # A freshly allocated tuple / output pair hashes slow for its launches
    # ~10-40 (0.55 against 0.69-0.72 of 8 TB/s before and after, in one
    # process, every pair: tools/rss_steady.py, profiles/r05/first/rss_steady.log),
    # exactly the bench's old window (5 warm-ups, then 20); the pair is
    # warmed past it first, so the line times the kernel's steady state.
    wall_h, ev_h = timed(torch, dist, eng, cgck,
                         lambda: eng.toeplitz(d.ptr, n, 12, 12, RSS_KEY, o.ptr, mask=0x7F),
                         steps, max(warmup, RSS_WARMUP))
    k_hash = eng.last_kernel
    # this run's first 4096 tuples and results, for the parity check of the checker leg
    host = np.zeros(4096 * 12, np.uint8)
    got = np.zeros(4096, np.uint32)
    d.download(host, stream=eng.stream)
    o.download(got, stream=eng.stream)
    eng.sync()
    d.free()
    o.free()

    nl, nf, qn = RSS_DST
    qi = plan["first"] // plan["n"] % qn
    key = np.frombuffer(RSS_KEY, np.uint8)
    prm = cgck.Engine.dst_params((0x0A000001, 0x0A000000 + nl), (0x0A010000, 0x0A010000 + nf - 1),
                                 0x5000, qn, qi, key)
    tuples = nl * nf * 60536
    out = cgck.DeviceBuffer(16 * tuples // qn * 2)
    cnt = cgck.DeviceBuffer(4)
    cap = tuples // qn * 2
    wall_d, ev_d = timed(torch, dist, eng, cgck, lambda: eng.dst_cache(prm, out.ptr, cap, cnt.ptr),
                         steps, warmup)
    k_dst = eng.last_kernel
    c = np.zeros(1, np.uint32)
    cnt.download(c, stream=eng.stream)
    eng.sync()
    out.free()
    cnt.free()
    return {"hash": (wall_h, ev_h, n, k_hash), "hash_sample": (host, got),
            "dst": (wall_d, ev_d, tuples, int(c[0]), k_dst)}


BURSTS = (32, 64, 128, 256, 512, 1024, 2048)   # receive / transmit burst sizes (netmap-like 2048 B slots)
BURST_LENS = (1500, 576, 64)   # MTU frames, con-gen's MTU-522 frames (con-gen.c:741) as 576 B, minimum frames


def bench_burst():
    """SURVEY §8(f) ranks 1 and 2 at the transport's burst granularity, through
    the C-ABI from C (tools/txburst.c): a BSD-verify cgck_desc_host per RX
    burst, the RX window (cgck_rx_begin + the stack's per-packet verify calls
    + cgck_rx_end), and the deferred TX window on a registered ring.
    Host-resident, so PCIe/latency bound: never `value`.  Returns all rows."""
    exe = os.path.join(ROOT, "tools", "txburst")
    if not os.path.exists(exe):
        return None
    r = run_pinned([exe, "0.15"], 240)
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-300:]}
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


def run_pinned(cmd, timeout, env=None):
    """A host harness as a child process pinned to one core (the middle CPU
    of this process's set, as cpu_burst pins the reference): the windows'
    per-burst cost is mostly misses on GPU-written lines, and unpinned runs
    of one build moved by up to 1.7x with the core they landed on
    (profiles/r05/loop3/ab_host/unpinned/)."""
    import subprocess
    cpus = sorted(os.sched_getaffinity(0))
    old = set(cpus)
    try:
        os.sched_setaffinity(0, {cpus[len(cpus) // 2]})  # the child inherits it
        return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                              env=dict(os.environ, **env) if env else None)
    finally:
        os.sched_setaffinity(0, old)


def bench_loop():
    """con-gen's worker loop at the checksum boundary (tools/txloop.c): both
    windows open across the iteration, bursts of 1..2048 64 B frames, the
    rest of the stack's work as 0 or 250 ns a frame or 50 us a burst; per
    form (the reference's own functions, pipelined, coalesced, synchronous)
    the worker's us per iteration, its wait and the post-to-verdict latency.
    Host-resident: never `value`.  Returns all rows."""
    exe = os.path.join(ROOT, "tools", "txloop")
    if not os.path.exists(exe):
        return None
    # mixes: verify only, replies in transmit slots, replies in the stack-local
    # packet (a full transmit ring: the synchronous calls),
    # and the full ring with the pending packets in a registered pool
    # (queued like ring slots, drained after their fill)
    r = run_pinned([exe, "0.1"], 300, env={"TXLOOP_MIXES": "0,1,2,3"})
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-300:]}
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


WORKERS = "1,4,12"   # worker threads on this GPU, each with its own pool, context and burst server (<= 12 a device)


def bench_workers():
    """con-gen's N-worker mode (con-gen.c:1062-1100) at the checksum
    boundary: tools/txloop's workers mode, each thread pinned to its own CPU
    with its own registered pool, context and burst server, 64-frame bursts,
    replies, 250 ns of stack work a frame, all threads in the same cell at
    once.  Host-resident: never `value`.  Returns per (N, form) the
    per-thread us per burst (median / p90 / max over the threads)."""
    exe = os.path.join(ROOT, "tools", "txloop")
    if not os.path.exists(exe):
        return None
    import subprocess
    env = dict(os.environ, TXLOOP_WORKERS=WORKERS)
    r = subprocess.run([exe, "0.1"], capture_output=True, text=True, timeout=300, env=env)
    if r.returncode != 0:
        return {"error": r.stderr.strip()[-300:]}
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return {"what": "per-thread us of the checksum path per 64 x 64 B burst with replies, 250 ns/frame of "
                    "stack work, N workers on one GPU each with its own ring, context and burst server "
                    "(tools/txloop workers mode)",
            "rows": [{k: x.get(k) for k in ("workers", "form", "us_per_burst", "us_iter_p90", "us_latency",
                                            "servers", "exact", "error") if k in x} for x in rows],
            "exact": all(x.get("exact") for x in rows)}


LOOP_FORMS = ("reference", "pipelined", "coalesced", "sync")


def loop_summary(rows):
    """Per (mix, stack budget): [burst, us per iteration of each form
    (LOOP_FORMS), the pipelined form's wait, the pipelined and coalesced
    forms' post-to-verdict latency]; per (mix, budget, form) the crossover
    burst (the smallest from which the form costs the worker less than the
    reference loop at every larger measured burst, None if never); the drain
    rule's lone-burst latency per burst."""
    if not isinstance(rows, list):
        return rows
    loop = [r for r in rows if r.get("mode") == "loop"]
    by = {(r["mix"], r["stack_ns_per_frame"], r["stack_us_fixed"], r["form"], r["burst"]): r for r in loop}
    cells = sorted({(r["mix"], r["stack_ns_per_frame"], r["stack_us_fixed"]) for r in loop})
    bursts = sorted({r["burst"] for r in loop})
    out = {"unit": "us of the worker thread's checksum path per burst processed",
           "cols": ["burst"] + [f"{f}_us" for f in LOOP_FORMS] + ["pipelined_wait_us", "pipelined_latency_us",
                                                                  "coalesced_latency_us"],
           "rows": {}, "crossover": {}, "exact": all(r.get("exact") for r in rows if "exact" in r)}
    for mix, ns, fx in cells:
        key = f"{mix}@{'%gus/burst' % fx if fx else '%gns/frame' % ns}"
        tab = []
        for b in bursts:
            g = lambda f, c="us_per_burst": by.get((mix, ns, fx, f, b), {}).get(c)
            tab.append([b] + [g(f) for f in LOOP_FORMS] + [g("pipelined", "us_wait"), g("pipelined", "us_latency"),
                                                         g("coalesced", "us_latency")])
        out["rows"][key] = tab
        cross = {}
        for fi, f in enumerate(LOOP_FORMS[1:], 2):
            first = None
            for row in reversed(tab):
                if row[1] is None or row[fi] is None or not row[fi] < row[1]:
                    break
                first = row[0]
            cross[f] = first
        out["crossover"][key] = cross
    out["lone_latency_us"] = {r["burst"]: r["us_latency"] for r in rows if r.get("mode") == "lone"}
    # a cell that processed no burst measured nothing (its figures are null,
    # tools/txloop.c): listed, never a crossover win, and the leg not exact
    empty = [f"{r['mix']}@{r['stack_ns_per_frame']:g}ns+{r['stack_us_fixed']:g}us/{r['form']}/{r['burst']}"
             f" (iters {r.get('iters')}, longest {r.get('max_iter_us')} us)"
             for r in loop if not r.get("bursts", 1)]
    out["empty_cells"] = empty
    if empty:
        out["exact"] = False
    return out


BURST_COLS = ["pkt_len", "burst", "rx_window_launch_us", "rx_window_server_us", "rx_window_pipelined_us",
              "tx_fill_launch_us", "tx_fill_server_us", "tx_fill_pipelined_us", "rx_ref_loop_us", "tx_ref_loop_us",
              "cpu_ref_us"]
# (column, txburst mode): each column is ONE routing, as measured (no per-cell
# minimum over routings): the launch path (no server open), the burst server
# opened wide (every burst of the cell goes to it), and the server with one
# burst in flight (host-thread-visible us per burst: post + wait + the
# stack's calls + end, the stack's other work overlapping the GPU)
BURST_MODES = (("rx_window_launch_us", "rx_window_registered"),
               ("rx_window_server_us", "rx_window_registered_server"),
               ("rx_window_pipelined_us", "rx_window_pipelined_registered_server"),
               ("tx_fill_launch_us", "tx_fill_registered"),
               ("tx_fill_server_us", "tx_fill_registered_server"),
               ("tx_fill_pipelined_us", "tx_fill_pipelined_registered_server"))
# the reference's own in_cksum / udp_cksum (oracle/_ref) in the same binary on
# the same ring: the RX loop saves / zeroes / computes / restores each field,
# the TX loop zeroes / computes / stores (one core, the harness's thread)
BURST_REF = (("rx_ref_loop_us", "rx_reference_loop"), ("tx_ref_loop_us", "tx_reference_loop"))


def burst_summary(rows, cpu):
    """At most 9 rows for the JSON line (columns BURST_COLS): per packet size
    and burst, the RX window and the TX window on a registered ring through
    each routing as measured, against the reference CPU loop over the same
    burst (us per burst)."""
    if not isinstance(rows, list):
        return rows
    by = {(r["mode"], r["pkt_len"], r["burst"]): r["us_median"] for r in rows}
    cpu_by = {(r["pkt_len"], r["burst"]): round(r["us_per_burst"], 2) for r in (cpu or {}).get("rows", [])}
    return [[ln, b] + [by.get((m, ln, b)) for _, m in BURST_MODES + BURST_REF] + [cpu_by.get((ln, b))]
            for ln in sorted(BURST_LENS) for b in (32, 256, 2048)]


def burst_crossover(rows, cpu):
    """Per packet length and routing, the smallest measured burst from which
    that routing beats the reference CPU loop over the same burst on one core,
    and stays ahead at every larger measured burst; None when it never wins up
    to max(BURSTS).  INTEGRATION.md quotes these as the threshold below which
    a window should not be opened."""
    if not isinstance(rows, list) or not cpu:
        return None
    by = {(r["mode"], r["pkt_len"], r["burst"]): r["us_median"] for r in rows}
    cpu_by = {(r["pkt_len"], r["burst"]): r["us_per_burst"] for r in cpu.get("rows", [])}
    res = {}
    for ln in sorted(BURST_LENS):
        cell = {}
        for col, mode in BURST_MODES:
            wins = [(mode, ln, b) in by and cpu_by.get((ln, b)) is not None and by[(mode, ln, b)] < cpu_by[(ln, b)]
                    for b in BURSTS]
            first = None
            for i in range(len(BURSTS) - 1, -1, -1):
                if not wins[i]:
                    break
                first = BURSTS[i]
            cell[col[:-3]] = first
        res[str(ln)] = cell
    return res


# SURVEY §8(d) parity gate: 100 % of the 64 B batch (configs[1]); a strided
# 1/64 sample over the WHOLE shard for 1500 B and IMIX (configs[2]-[4])
CHECK_EVERY = {"64": 1, "1500": 64, "imix": 64}


def checker_leg(res, plan, cgck):
    """Parity of this rank's outputs of this run against the oracle (the
    oracle is only the checker here), on its own shard (seed 0xC0C0 + rank):
    every packet of the 64 B batch, every 64th packet across the whole 1500 B
    and IMIX batches (CHECK_EVERY), and the first 4096 hashed tuples.
    Returns {workload: [checked, mismatches]}."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    P = oracle.port()
    par = {}
    for key, size in (("1500", 1500), ("64", 64)):
        if key in res:
            o = res[key]["out"]
            bad, chk = P.check_synth_strided(len(o), size, size, plan["seed"], cgck.GEN_BOTH, o,
                                             CHECK_EVERY[key])
            par[key] = [chk, bad]
    if "imix" in res:
        o, ou, orr = res["imix"]["out"]
        bad, chk = P.check_synth_imix(len(o), plan["seed"], cgck.GEN_BOTH, o, CHECK_EVERY["imix"])
        par["imix"] = [chk, bad]
        bad, chk = P.check_synth_imix(len(ou), plan["seed"], cgck.GEN_BOTH, ou, CHECK_EVERY["imix"])
        par["imix_unhinted"] = [chk, bad]
        bad, chk = P.check_synth_ring(len(orr), RING_SLOT, RING_L3, plan["seed"], cgck.GEN_BOTH, orr,
                                      CHECK_EVERY["imix"])
        par["imix_ring"] = [chk, bad]
    if "rss" in res:
        host, got = res["rss"]["hash_sample"]
        exp = P.toeplitz_batch(host, 4096, 12, 12, np.frombuffer(RSS_KEY, np.uint8), mask=0x7F)
        par["rss"] = [4096, int(np.count_nonzero(got != exp))]
    return par


def cpu_burst():
    """The reference's per-packet pair (in_cksum(ip, 20) + udp_cksum(ip, len - 20),
    the recompute that both verify and fill perform) over one burst of the same
    ring layout, on one pinned core: microseconds per burst."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    P = oracle.port()
    R = oracle.reference()
    fin, fudp = (R or P).fn_pointers()
    cpus = sorted(os.sched_getaffinity(0))
    old = set(cpus)
    rows = []
    try:
        os.sched_setaffinity(0, {cpus[len(cpus) // 2]})
        for ln in BURST_LENS:
            ring = P.stream_bytes(0, max(BURSTS) * 2048, SEED)
            P.stamp_strided(ring[14:], max(BURSTS) - 1, 2048, ln)
            for b in BURSTS:
                m = min(b, max(BURSTS) - 1)
                reps = max(1, int(2e6 // (m * ln)))
                sec, _ = P.cpu_bench(fin, fudp, ring[14:], m, 2048, ln, threads=1, reps=reps)
                rows.append({"pkt_len": ln, "burst": b, "us_per_burst": sec / reps * 1e6 * b / m,
                             "mpkt_s": m * reps / sec / 1e6})
    finally:
        os.sched_setaffinity(0, old)
    return {"unit": "us per burst", "cores": 1, "kind": "reference" if R else "port",
            "sample": "in_cksum(ip,20)+udp_cksum(ip,len-20) per packet over one burst of 2048 B "
                      "slots (IPv4 at +14), cache-warm", "rows": rows}


def cpu_rss(seconds):
    """The reference loop (con-gen.c:291-360, restated in oracle/rss_oracle.c)
    calling the REFERENCE's own rss_hash4 (oracle/_ref/libref_rss.so) when
    built, on one pinned core: 1 laddr x 16 faddrs x 60536 ports, 8 queues."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    P = oracle.port()
    R = oracle.reference_rss()
    fn = R.fn_rss_hash4() if R else None
    key = np.frombuffer(RSS_KEY, np.uint8)
    cpus = sorted(os.sched_getaffinity(0))
    old = set(cpus)
    tuples, reps, t = 16 * 60536, 0, 0.0
    try:
        os.sched_setaffinity(0, {cpus[len(cpus) // 2]})
        while t < seconds:
            t0 = time.perf_counter()
            P.dst_cache(0x0A000001, 0x0A000001, 0x0A010000, 0x0A01000F, 0x5000, 8, 3, key,
                        1 << 30, hash_fn=fn)
            t += time.perf_counter() - t0
            reps += 1
    finally:
        os.sched_setaffinity(0, old)
    return {"value": tuples * reps / t / 1e9, "unit": "Gtuple/s", "cores": 1,
            "kind": "reference" if R else "port",
            "sample": f"dst-cache loop over 1 laddr x 16 faddrs x 60536 ports (968576 tuples), "
                      f"8 queues, {reps} passes, {t:.1f} s on 1 pinned core"}


def cpu_baseline(seconds):
    """The reference's checksum loop on this box's host cores (rank 0, N = 1):
    in_cksum(ip, 20) + udp_cksum(ip, 1480) per 1500 B packet, dense stride,
    cache-cold (sample larger than the LLC), one pinned core."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    P = oracle.port()
    R = oracle.reference()
    fin, fudp = (R or P).fn_pointers()
    kind = "reference" if R else "port"
    n = 262144
    buf = np.zeros(n * 1500, np.uint8)
    for k in range(0, n, 4096):   # same synthetic bytes as the device batch
        m = min(4096, n - k)
        blk = P.stream_bytes(k * 1500, m * 1500, SEED)
        buf[k * 1500:(k + m) * 1500] = blk
    P.stamp_strided(buf, n, 1500, 1500)
    cpus = sorted(os.sched_getaffinity(0))
    old = set(cpus)
    try:
        os.sched_setaffinity(0, {cpus[len(cpus) // 2]})
        sec, _ = P.cpu_bench(fin, fudp, buf, n, 1500, 1500, threads=1, reps=1)
        reps = max(1, int(seconds / max(sec, 1e-3)))
        sec, _ = P.cpu_bench(fin, fudp, buf, n, 1500, 1500, threads=1, reps=reps)
    finally:
        os.sched_setaffinity(0, old)
    rate = n * reps / sec
    # the box's CPU share for one GPU (OMP_NUM_THREADS is 16 there)
    allc = min(len(cpus), int(os.environ.get("OMP_NUM_THREADS", "16") or 16), 16)
    sec_all, _ = P.cpu_bench(fin, fudp, buf, n, 1500, 1500, threads=allc, reps=max(1, reps // 4))
    rate_all = n * max(1, reps // 4) / sec_all
    return {
        "value": rate / 1e9, "unit": "Gpkt/s", "cores": 1, "kind": kind,
        "sample": f"{n} x 1500 B packets (393 MB, cache-cold), in_cksum(ip,20)+udp_cksum(ip,1480) "
                  f"each, {reps} passes, {sec:.1f} s on 1 pinned core",
        "gbps": rate * 1500 / 1e9,
        "all_cores": {"value": rate_all / 1e9, "cores": allc, "gbps": rate_all * 1500 / 1e9},
    }


def cpu_baseline_64(seconds):
    """BASELINE configs[0]: 1M x 64 B IPv4+TCP packets through the reference's
    checksum loop (in_cksum(ip, 20) + udp_cksum(ip, 44) each) on one pinned
    host core, same synthetic bytes as the device batch."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    P = oracle.port()
    R = oracle.reference()
    fin, fudp = (R or P).fn_pointers()
    n = 1 << 20
    buf = P.stream_bytes(0, n * 64, SEED)
    P.stamp_strided(buf, n, 64, 64)
    cpus = sorted(os.sched_getaffinity(0))
    old = set(cpus)
    try:
        os.sched_setaffinity(0, {cpus[len(cpus) // 2]})
        sec, _ = P.cpu_bench(fin, fudp, buf, n, 64, 64, threads=1, reps=1)
        reps = max(1, int(seconds / max(sec, 1e-3)))
        sec, _ = P.cpu_bench(fin, fudp, buf, n, 64, 64, threads=1, reps=reps)
    finally:
        os.sched_setaffinity(0, old)
    rate = n * reps / sec
    return {"value": rate / 1e9, "unit": "Gpkt/s", "cores": 1, "kind": "reference" if R else "port",
            "sample": f"BASELINE configs[0]: {n} x 64 B packets (64 MB), in_cksum(ip,20)+udp_cksum(ip,44) "
                      f"each, {reps} passes, {sec:.1f} s on 1 pinned core",
            "gbps": rate * 64 / 1e9}


TRAFFIC_SOURCE = ("profiles/pmc_latest.json: FETCH_SIZE x 2 + WRITE_SIZE per launch from separate "
                  "rocprofv3 --pmc passes of this bench (tools/gpu_prof.sh), not measured in this run")
TRAFFIC_LIVE = ("this run: rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE, each a pass of its own over "
                "tools/one_workload.py (the same batch and kernel, 3 launches, a child process on this box "
                "after the timed region); bytes = (2 x FETCH_SIZE + WRITE_SIZE) KB x 1024, the median per "
                "dispatch.  The x 2: on gfx950 FETCH_SIZE = TCC_EA0_RDREQ x 64 B while each request of a "
                "wide streaming read moves 128 B (/opt/skills/guides/MI355X_MICROARCH.md, HBM/rocprofv3 "
                "section; in this repo profiles/r02/state64/README.md: TCC_EA0_RDREQ per 1 GiB 64 B-batch "
                "dispatch = 8.39M = the batch's bytes / 128, and the doubled FETCH_SIZE of each workload "
                "matches its algorithmic read bytes to 0.01-1 %, profiles/pmc_latest.json)")


def pmc_traffic_live(kernels):
    """HBM bytes per launch of each workload's kernel, measured on this box
    now: two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: together they
    exceed the four TCC counters of one pass) over one_workload.py per
    workload.  {workload: bytes} for the workloads whose passes succeeded."""
    import csv
    import glob
    import shutil
    import statistics
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return {}
    env = dict(os.environ, TMPDIR="/tmp")
    res = {}
    for w, kernel in kernels.items():
        got = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = tempfile.mkdtemp(prefix="cgck_pmc_", dir="/tmp")
            cmd = ["rocprofv3", "--pmc", ctr, "-d", d, "-o", "run", "--output-format", "csv", "--",
                   sys.executable, os.path.join(ROOT, "tools", "one_workload.py"), w, "--launches", "3"]
            try:
                subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, timeout=120)
                vals = []
                for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
                    for r in csv.DictReader(open(f)):
                        if r.get("Counter_Name") == ctr and kernel in r.get("Kernel_Name", ""):
                            vals.append(float(r["Counter_Value"]))
                if vals:
                    got[ctr] = statistics.median(vals) * 1024
            except (OSError, subprocess.SubprocessError, ValueError, KeyError):
                pass
            finally:
                shutil.rmtree(d, ignore_errors=True)
        if len(got) == 2:
            res[w] = 2 * got["FETCH_SIZE"] + got["WRITE_SIZE"]
    return res


def load_traffic(key="1500", kernel=None):
    """Per-launch HBM bytes of a workload's kernel from the committed PMC
    summary (profiles/pmc_latest.json, written by tools/pmc_traffic.py from
    separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench);
    None when the summary was taken on another kernel than this run's."""
    p = os.path.join(ROOT, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if kernel and d.get("kernels", {}).get(key) not in (None, kernel):
        return None
    return d.get(f"bytes_per_launch_{key}")


def roofline(n, size, ev_ms, kernel, traffic_key, extra_bytes=0, live=None):
    """HBM roofline of one workload's kernel: algorithmic bytes per launch
    (n x (L + 4) [+ descriptors]) over its HIP-event time per launch.
    traffic: the PMC bytes per launch measured in this run (live), else the
    committed summary of the same kernel."""
    algo = n * (size + 4) + extra_bytes
    ach = algo / (ev_ms * 1e-3)
    if live and traffic_key in live:
        traffic, src = live[traffic_key], TRAFFIC_LIVE
    else:
        traffic, src = load_traffic(traffic_key, kernel), TRAFFIC_SOURCE
    return {"bound": "hbm", "achieved": ach / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s",
            "frac": ach / HBM_PEAK, "traffic": traffic, "kernel": kernel,
            # the same launch in HBM bytes (PMC): what the memory system moved per second
            "hbm_frac": traffic / (ev_ms * 1e-3) / HBM_PEAK if traffic else None,
            "algorithmic_bytes_per_launch": algo, "kernel_ms_hip_events": ev_ms,
            "traffic_over_algorithmic": traffic / algo if traffic else None, "traffic_source": src}


def main():
    args = parse()
    how, world = launch_decision(args.gpus, os.environ)
    if how == "spawn":   # before torch is imported: nothing here has touched the GPU
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    import torch   # first: the process then shares torch's HIP runtime
    dist = Dist()
    assert dist.world == world
    # one rank per GPU; a rehearsal on fewer GPUs must say so
    dev = device_for(dist.local, dist.world, torch.cuda.device_count(), args.allow_shared_devices)
    torch.cuda.set_device(dev)
    import cgck
    eng = cgck.Engine(dev)
    plan = shard_plan(dist.rank, dist.world, args.packets)
    n = plan["n"]
    res = {}

    if args.only in (None, "1500"):
        wall, ev_ms, o, k = bench_strided(torch, dist, eng, cgck, n, 1500, plan, args.steps, args.warmup)
        res["1500"] = {"wall": wall, "ev": ev_ms, "out": o, "kernel": k}
    if not args.no_extra and args.only in (None, "64"):
        wall, ev_ms, o, k = bench_strided(torch, dist, eng, cgck, n, 64, plan, args.steps, args.warmup)
        res["64"] = {"wall": wall, "ev": ev_ms, "out": o, "kernel": k}
    if not args.no_extra and args.only in (None, "imix"):
        wall, ev_ms, nbytes, o, k, unh, ring = bench_imix(torch, dist, eng, cgck, n, plan, args.steps, args.warmup)
        res["imix"] = {"wall": wall, "ev": ev_ms, "bytes": nbytes, "out": o, "kernel": k, "unhinted": unh,
                       "ring": ring}
    if not args.no_rss and args.only in (None, "rss"):
        res["rss"] = bench_rss(torch, dist, eng, cgck, plan, args.steps, args.warmup)

    # every rank checks its own shard; the totals are summed over ranks
    par = checker_leg(res, plan, cgck)
    parity = {k: {"checked": int(dist.sum(v[0])), "mismatches": int(dist.sum(v[1])), "ranks": dist.world}
              for k, v in sorted(par.items())}
    devices = dist.gather({"rank": dist.rank, "local_rank": dist.local, "device": dev,
                           "pci_bus": torch.cuda.get_device_properties(dev).pci_bus_id
                           if hasattr(torch.cuda.get_device_properties(dev), "pci_bus_id") else None})

    burst = loop = workers = None
    if dist.rank == 0 and dist.world == 1 and not args.no_burst and args.only is None:
        burst = bench_burst()
        loop = bench_loop()
        workers = bench_workers()
    cpu = cpu_r = cpu_64 = cpu_b = None
    if dist.rank == 0 and dist.world == 1 and not args.no_cpu:
        if burst:
            cpu_b = cpu_burst()
        cpu = cpu_baseline(args.cpu_seconds)
        if "64" in res:
            cpu_64 = cpu_baseline_64(min(3.0, args.cpu_seconds))
        if "rss" in res:
            cpu_r = cpu_rss(min(3.0, args.cpu_seconds))
    live = {}
    if dist.rank == 0 and dist.world == 1 and not args.no_pmc:
        kern = {k: res[k]["kernel"] for k in ("1500", "64", "imix") if k in res}
        if "imix" in res:
            kern["ring"] = res["imix"]["ring"]["kernel"]
        live = pmc_traffic_live(kern)
    dist.barrier()

    if dist.rank == 0:
        W = dist.world
        K = args.steps
        shared = len({d["device"] for d in devices}) < W
        out = {"metric": METRIC, "unit": "Gpkt/s", "n_gpus": W, "steps": K, "warmup": args.warmup,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u16",
               "data": "synthetic (device-generated splitmix64 IPv4+TCP packets, SURVEY §8(d))"}
        if shared:
            out["shared_devices"] = "REHEARSAL: ranks share GPUs; not an N-GPU measurement"
        if "1500" in res:
            r = res["1500"]
            gpkt = n * W * K / r["wall"] / 1e9
            out.update({
                "value": gpkt, "ms_per_step": r["wall"] / K * 1e3,
                "config": {"workload": f"{n} x 1500 B IPv4+TCP per GPU, dense stride 1500, "
                                       "ip_cksum + tcp_cksum per packet (BASELINE configs[2]; "
                                       "configs[4] at 8 GPUs)",
                           "packets_per_gpu": n, "packet_bytes": 1500, "parallelism": f"batch-split x{W}",
                           "gb_s": gpkt * 1500, "devices": [d["device"] for d in devices]},
                "roofline": roofline(n, 1500, r["ev"], r["kernel"], "1500", live=live),
            })
        if "64" in res:
            r = res["64"]
            gpkt = n * W * K / r["wall"] / 1e9
            out.update({"value_64B": gpkt, "gb_s_64B": gpkt * 64, "ms_per_step_64B": r["wall"] / K * 1e3,
                        "config_64B": f"{n} x 64 B IPv4+TCP per GPU, dense stride 64 (BASELINE configs[1])",
                        "roofline_64B": roofline(n, 64, r["ev"], r["kernel"], "64", live=live)})
        if "imix" in res:
            r = res["imix"]
            gpkt = n * W * K / r["wall"] / 1e9
            # algorithmic bytes: the frames, 12 B of descriptor and 4 B of output per packet
            out.update({"value_imix": gpkt, "gb_s_imix": r["bytes"] * W * K / r["wall"] / 1e9,
                        "ms_per_step_imix": r["wall"] / K * 1e3,
                        "config_imix": f"{n} IMIX packets per GPU (64/576/1500 at 7:4:1, 12-byte "
                                       "descriptors; BASELINE configs[3]), frames back to back: "
                                       "cgck_set_desc_layout(CGCK_LAYOUT_PACKED)",
                        "roofline_imix": roofline(n, 0, r["ev"], r["kernel"], "imix", r["bytes"] + 12 * n,
                                                  live=live),
                        "imix_without_layout_hint": r["unhinted"], "imix_ring": r["ring"]})
            rg = r["ring"]
            if live.get("ring"):
                # ring slots cost whole lines: a frame at +14 reads 128 B for 64 B, 640 B for
                # 576 B, 1536 B for 1500 B (1.174x the IMIX cycle), so the ring's HBM bytes are
                # its PMC traffic, not the algorithmic bytes
                rg["traffic"] = live["ring"]
                rg["traffic_over_algorithmic"] = live["ring"] / (r["bytes"] + 16 * n)
                rg["hbm_frac"] = live["ring"] / (rg["kernel_ms"] * 1e-3) / HBM_PEAK
                rg["traffic_source"] = TRAFFIC_LIVE
        out["parity"] = parity
        if cpu:
            out["cpu_baseline"] = cpu
        if cpu_64:
            out["cpu_baseline_cfg0"] = cpu_64
        extra = {}
        if "rss" in res:
            wall_h, ev_h, nt, k_hash = res["rss"]["hash"]
            wall_d, ev_d, td, written, k_dst = res["rss"]["dst"]
            ach = nt * 16 / (ev_h * 1e-3)
            extra["rss_hash"] = {
                "workload": f"{nt} dense 12-byte tuples per GPU, rss_hash4 (mask 0x7F)", "kernel": k_hash,
                "gtuple_s": nt * W * K / wall_h / 1e9, "kernel_ms": ev_h, "achieved_gbs": ach / 1e9,
                "hbm_frac": ach / HBM_PEAK, "algorithmic_bytes_per_launch": nt * 16,
                "traffic": load_traffic("rss_hash")}
            extra["dst_cache"] = {
                "workload": f"thread_init_dst_cache over {td} tuples per GPU ({RSS_DST[0]} laddrs x "
                            f"{RSS_DST[1]} faddrs x 60536 ports, {RSS_DST[2]} queues)", "kernel": k_dst,
                "gtuple_s": td * W * K / wall_d / 1e9, "kernel_ms": ev_d, "entries_written": written}
            if cpu_r:
                extra["dst_cache"]["cpu_baseline"] = cpu_r
        if burst:
            path = os.path.join(ROOT, "gpurun_out", "bench_burst.json")
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "w") as f:
                    json.dump({"rows": burst, "cpu_baseline": cpu_b, "loop_rows": loop}, f, indent=0)
            except OSError:
                path = None
            extra["burst"] = {"what": "us per burst, 2048 B ring slots registered with cgck_host_register, "
                                      "from C (tools/txburst.c): RX window and TX window through the launch "
                                      "path, the burst server, and the server with one burst in flight "
                                      "(host-thread-visible us, the stack's other work overlapping); "
                                      "cpu_ref = the reference in_cksum+udp_cksum per packet, 1 core",
                              "cols": BURST_COLS, "rows": burst_summary(burst, cpu_b),
                              "crossover_burst": burst_crossover(burst, cpu_b),
                              "all_rows": path and "gpurun_out/bench_burst.json",
                              "loop": loop_summary(loop), "workers": workers}
        if extra:
            out["extra"] = extra
        if "value" not in out:   # --only 64 / imix / rss profiling runs
            if "value_64B" in out:
                out["value"], out["config"] = out["value_64B"], {"workload": "64B"}
            elif "value_imix" in out:
                out["value"], out["config"] = out["value_imix"], {"workload": "imix"}
            else:
                out["value"], out["config"] = extra["rss_hash"]["gtuple_s"], {"workload": "rss_hash"}
        print(json.dumps(out), flush=True)
    eng.close()
    dist.close()


if __name__ == "__main__":
    main()
