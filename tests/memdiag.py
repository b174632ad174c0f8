"""Host-memory diagnostics for the registered-ring tests: which mapping a
ring lies in (/proc/self/smaps: its VMA flags, transparent huge pages) and
what the kernel did to pages meanwhile (/proc/vmstat: THP faults, splits and
collapses, page migrations), so a failure on the GPU box says whether the
ring's pages were remapped under the GPU."""

VMSTAT_KEYS = ("thp_fault_alloc", "thp_split_pmd", "thp_collapse_alloc", "pgmigrate_success",
               "numa_pages_migrated", "compact_success")


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


def vmstat_delta(a, b):
    return {k: b[k] - a.get(k, 0) for k in b if b[k] != a.get(k, 0)}


def vma_info(addr, nbytes):
    """The smaps entries of the mappings that [addr, addr + nbytes) touches:
    range, VmFlags (hg = MADV_HUGEPAGE, nh = MADV_NOHUGEPAGE, lo = mlocked),
    AnonHugePages and THPeligible."""
    out = []
    try:
        with open("/proc/self/smaps") as f:
            cur = None
            for line in f:
                head = line.split()
                if "-" in head[0] and len(head) >= 5 and ":" not in head[0]:
                    lo, hi = (int(x, 16) for x in head[0].split("-"))
                    cur = {"range": head[0], "name": head[5] if len(head) > 5 else ""} \
                        if lo < addr + nbytes and hi > addr else None
                    if cur is not None:
                        out.append(cur)
                elif cur is not None and head[0] in ("AnonHugePages:", "THPeligible:", "VmFlags:", "Rss:"):
                    cur[head[0][:-1]] = " ".join(head[1:])
    except OSError as e:
        return [{"error": str(e)}]
    return out


def dump_failure(what, **arrays):
    """Save a failing request's arrays under gpurun_out/ (merged back from the
    GPU box) for offline analysis; returns the path, or None."""
    import os
    import re

    import numpy as np
    root = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    d = os.path.join(root, "gpurun_out", "failures")
    try:
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, re.sub(r"[^A-Za-z0-9_]+", "_", what)[:80] + f"_{os.getpid()}.npz")
        np.savez_compressed(path, **arrays)
        return os.path.relpath(path, root)
    except OSError:
        return None


def in_brk_heap(addr, nbytes):
    """Does [addr, addr + nbytes) touch the brk heap ([heap] in /proc/self/maps)?"""
    with open("/proc/self/maps") as f:
        for line in f:
            if "[heap]" in line:
                lo, hi = (int(x, 16) for x in line.split()[0].split("-"))
                if lo < addr + nbytes and hi > addr:
                    return True
    return False
