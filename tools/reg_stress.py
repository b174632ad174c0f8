"""Diagnostic for the registered-ring burst-server path:
replay test_burst_server_wide's registered sequence — a fresh ring per batch
size, cgck_host_register, GEN / FILL / VERIFY through a 32-workgroup server,
cgck_host_unregister, free — for a bounded time, and on every mismatch print
which packets, which server slice, the ring's address and size, and what the
kernel's memory saw around the request (/proc/vmstat deltas: NUMA-balancing
hinting faults and page migrations, THP collapses, compaction).

usage: python tools/reg_stress.py [seconds] [mode] [libcgck.so]
  mode "plain": numpy rings as the test allocates them
  mode "lock":  the same rings mlock'ed and MADV_NOHUGEPAGE before registering
  mode "heap":  plain rings after priming the heap as a long test process does
                (a 30 MB array freed raises glibc's mmap threshold, then an 8 MB
                array comes from the heap and numpy marks it MADV_HUGEPAGE)
  mode "mmap":  each ring its own anonymous mmap, MADV_NOHUGEPAGE
"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "con-gen_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import cgck  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import random_batch  # noqa: E402

VMSTAT_KEYS = ("numa_hint_faults", "numa_pages_migrated", "pgmigrate_success", "pgmigrate_fail",
               "thp_collapse_alloc", "thp_fault_alloc", "compact_migrate_scanned", "compact_success",
               "thp_split_pmd", "pgfault")


def vmstat():
    d = {}
    try:
        with open("/proc/vmstat") as f:
            for line in f:
                k, v = line.split()
                if k in VMSTAT_KEYS:
                    d[k] = int(v)
    except OSError:
        pass
    return d


def vdelta(a, b):
    return {k: b[k] - a.get(k, 0) for k in b if b[k] != a.get(k, 0)}


def sysinfo():
    out = {}
    for p in ("/proc/sys/kernel/numa_balancing", "/sys/kernel/mm/transparent_hugepage/enabled",
              "/sys/kernel/mm/transparent_hugepage/defrag",
              "/sys/kernel/mm/transparent_hugepage/khugepaged/defrag",
              "/proc/sys/vm/compact_unevictable_allowed"):
        try:
            with open(p) as f:
                out[p] = f.read().strip()
        except OSError as e:
            out[p] = f"({e.strerror})"
    import resource
    out["RLIMIT_MEMLOCK"] = resource.getrlimit(resource.RLIMIT_MEMLOCK)
    out["numa_nodes"] = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")]) \
        if os.path.isdir("/sys/devices/system/node") else "?"
    out["affinity"] = len(os.sched_getaffinity(0))
    return out


libc = ctypes.CDLL(None, use_errno=True)
MADV_NOHUGEPAGE = 15


def burst_wgs(n, K, per=64):
    return 1 if n <= 64 else min((n + per - 1) // per, K)


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 60
    mode = sys.argv[2] if len(sys.argv) > 2 else "plain"
    print("sysinfo", sysinfo(), flush=True)
    L = cgck.load(sys.argv[3] if len(sys.argv) > 3 else None)
    print("library", cgck.LIB_PATH if len(sys.argv) <= 3 else sys.argv[3], flush=True)
    P = oracle.port()
    eng = cgck.Engine(0)
    max_pkts, K = 4096, 32
    eng.burst_open(max_pkts=max_pkts, max_bytes=4 << 20)
    names = {cgck.GEN_BOTH: "GEN", cgck.FILL_BOTH: "FILL", cgck.VERIFY_BSD: "VBSD"}
    if mode == "heap":
        a = np.ones(30 << 20, np.uint8)
        del a
        b = np.ones(8 << 20, np.uint8)
        del b
    import mmap as _mmap
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import memdiag
    t_end = time.time() + seconds
    cycle = requests = bad_requests = 0
    reg_ms, unreg_ms = [], []   # wall time of cgck_host_register / _unregister with the server open
    raw = None
    try:
        while time.time() < t_end:
            for max_len in (80, 600):
                for npk in (64, 65, 130, 2047, 2048, 4096):
                    rng = np.random.default_rng(77 + npk + max_len + 1000 * cycle)
                    buf, desc = random_batch(rng, npk, max_len)
                    size = (len(buf) + 4095) // 4096 * 4096
                    ring = None
                    if mode == "mmap":
                        raw = _mmap.mmap(-1, size, flags=_mmap.MAP_PRIVATE | _mmap.MAP_ANONYMOUS)
                        ring = np.frombuffer(raw, np.uint8)
                        libc.madvise(ctypes.c_void_p(ring.ctypes.data), ctypes.c_size_t(size), MADV_NOHUGEPAGE)
                    else:
                        raw = np.zeros(size + 4096, np.uint8)
                        off = (-raw.ctypes.data) % 4096
                        ring = raw[off:off + size]
                    if cycle == 0 and npk == 4096:
                        print("ring mapping", memdiag.vma_info(ring.ctypes.data, size), flush=True)
                    if mode == "lock":
                        if libc.madvise(ctypes.c_void_p(ring.ctypes.data), ctypes.c_size_t(size), MADV_NOHUGEPAGE):
                            print("madvise errno", ctypes.get_errno())
                        if libc.mlock(ctypes.c_void_p(ring.ctypes.data), ctypes.c_size_t(size)):
                            print("mlock errno", ctypes.get_errno())
                    t_reg = time.perf_counter()
                    assert L.cgck_host_register(ring.ctypes.data, size) == 0
                    reg_ms.append((time.perf_counter() - t_reg) * 1e3)
                    try:
                        for flags in (cgck.GEN_BOTH, cgck.FILL_BOTH, cgck.VERIFY_BSD):
                            ref = buf.copy()
                            exp, ever = P.batch_desc(ref, desc.view(np.uint8), len(desc), flags)
                            ring[:len(buf)] = buf
                            got = ring[:len(buf)]
                            out = np.zeros(len(desc), np.uint32)
                            ver = np.zeros(len(desc), np.uint8)
                            v0 = vmstat()
                            err = ""
                            try:
                                eng.desc_host(got, desc, flags, out, ver)
                            except cgck.CgckError as e:
                                err = str(e)
                            v1 = vmstat()
                            requests += 1
                            bad = np.nonzero((out != exp) | (ver != ever))[0]
                            bytes_bad = np.nonzero(got != ref)[0]
                            if len(bad) or len(bytes_bad) or err:
                                bad_requests += 1
                                W = burst_wgs(npk, K)
                                sl = sorted({int(np.searchsorted([npk * j // W for j in range(1, W + 1)], int(i),
                                                                  side="right")) for i in bad})
                                fo = desc["frame_off"].astype(np.int64) + desc["l3_off"]
                                print(f"MISMATCH cycle {cycle} npk {npk} max_len {max_len} {names[flags]} err '{err}' "
                                      f"W {W} bad {len(bad)} first {bad[:6].tolist()} last {bad[-6:].tolist()} "
                                      f"slices {sl[:12]} bytes_bad {len(bytes_bad)} ring {ring.ctypes.data:#x} "
                                      f"size {size} bad_offsets {fo[bad[:4]].tolist()} "
                                      f"got {out[bad[:3]].tolist()} want {exp[bad[:3]].tolist()} "
                                      f"vmstat {vdelta(v0, v1)} "
                                      f"bytes got {got[bytes_bad[:6]].tolist()} want {ref[bytes_bad[:6]].tolist()} "
                                      f"pages {sorted(set((bytes_bad // 4096).tolist()))[:12]} "
                                      f"mapping {memdiag.vma_info(ring.ctypes.data, size)}", flush=True)
                    finally:
                        t_unreg = time.perf_counter()
                        assert L.cgck_host_unregister(ring.ctypes.data) == 0
                        unreg_ms.append((time.perf_counter() - t_unreg) * 1e3)
                        if mode == "lock":
                            libc.munlock(ctypes.c_void_p(ring.ctypes.data), ctypes.c_size_t(size))
                        # (an mmap'ed ring is unmapped when its last view goes)
            cycle += 1
            print(f"cycle {cycle} requests {requests} bad {bad_requests} vmstat {vmstat()}", flush=True)
    finally:
        eng.burst_close()
    import statistics
    print(f"register ms median {statistics.median(reg_ms):.3f} max {max(reg_ms):.3f}; unregister ms median "
          f"{statistics.median(unreg_ms):.3f} max {max(unreg_ms):.3f} (server open, idle 200 ms)", flush=True)
    print(f"DONE mode {mode} cycles {cycle} requests {requests} bad_requests {bad_requests}", flush=True)
    return 1 if bad_requests else 0


if __name__ == "__main__":
    sys.exit(main())
