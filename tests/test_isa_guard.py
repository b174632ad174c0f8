"""CPU-side ISA guard (tools/isa_guard.py) for the product kernels whose
pipelines rest on hand-counted `s_waitcnt vmcnt(N)`.  clang emits the device
assembly of cgck_dense.hip / cgck_lane.hip for gfx950 here (no GPU); the test
asserts, per kernel:

  * no scratch: private segment 0, no VGPR spills, no scratch_* instruction;
  * VGPRs within the launch shape's budget (waves per SIMD the launcher runs);
  * the steady state of the loop holding the counted waits: along every path
    from one counted wait to the next, exactly the DMA instructions the wait
    constants assume (dstr: kDsS = 6 per step, cgck_dense.hip:49,258-260;
    lpd: 4 per step, cgck_lane.hip:374-408; lpw: kLpwDma + 1 = 9 per round,
    cgck_lane.hip:1533-1535, or two rounds when the step's first window was
    issued at the step's top), no other load, and the flush's stores as
    designed (lpd C / 4 = 8 per chunk, lpw one deferred store per lane);
  * the prologue: D (dstr 3, lpd 2) steps of DMA before the first wait.

An extra VMEM instruction the compiler adds inside a counted region (a spill,
a hoisted load) or a DMA it drops changes these counts; the last two tests
show the guard failing on exactly that, injected into the assembly text."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_guard  # noqa: E402

CSRC = os.path.join(ROOT, "con-gen_amd", "csrc")
INC = os.path.join(ROOT, "include")

# kernel: (source, mangled-name fragment, VGPR budget, steady DMA counts,
#          prologue DMA counts, flush store terms that must occur)
KERNELS = {
    # 128 threads, 8 workgroups per CU: 4 waves per SIMD -> 128 VGPRs
    "dstr": ("cgck_dense.hip", "dstr_kernelILi3ELi16ELb1ELi0E", 128, {6}, {18}, {0}),
    # 64 threads, 8 workgroups per CU: 2 waves per SIMD -> 256 VGPRs
    "lpd": ("cgck_lane.hip", "lpd_kernelILi2ELi32ELi2E", 256, {4}, {8}, {0, 8}),
    # one wave per workgroup, 8 per CU: 2 waves per SIMD -> 256 VGPRs
    "lpw": ("cgck_lane.hip", "lpw_kernelILb1ELi4ELb0E", 256, {9, 18}, set(), {0, 1}),
}


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    d = tmp_path_factory.mktemp("isa")
    out = {}
    for src in {v[0] for v in KERNELS.values()}:
        out[src] = isa_guard.device_asm(os.path.join(CSRC, src), str(d / (src + ".s")), include_dirs=(INC,))
    return out


def verify(text, part, budget, dma, prologue, stores):
    r = isa_guard.check(text, part)
    m = r["meta"]
    problems = []
    if m.get("private_segment_fixed_size") != 0 or m.get("vgpr_spill_count") != 0 or r["scratch_ops"]:
        problems.append(f"scratch: {m.get('private_segment_fixed_size')} B private, "
                        f"{m.get('vgpr_spill_count')} VGPR spills, {r['scratch_ops']} scratch ops")
    if m.get("uses_dynamic_stack") not in (None, "false"):
        problems.append("dynamic stack")
    if not m.get("vgpr_count") or m["vgpr_count"] > budget:
        problems.append(f"{m.get('vgpr_count')} VGPRs > {budget}")
    if not r["steady"]:
        problems.append("no counted wait found")
    seen_stores = set()
    for n, lab, segs in r["steady"]:
        if not segs:
            problems.append(f"vmcnt({n}) at {lab}: no path reaches another counted wait")
        for d, ld, st in segs:
            if d not in dma:
                problems.append(f"vmcnt({n}) at {lab}: {d} DMA between counted waits (expected {sorted(dma)})")
            if ld:
                problems.append(f"vmcnt({n}) at {lab}: {ld} other load(s) between counted waits")
            seen_stores.add(st)
    if not stores <= seen_stores:
        problems.append(f"flush store terms {sorted(stores)} not all found ({sorted(seen_stores)[:12]})")
    if prologue and set(r["entry_dma"]) != prologue:
        problems.append(f"prologue DMA {r['entry_dma']} (expected {sorted(prologue)})")
    return problems


@pytest.mark.parametrize("kernel", sorted(KERNELS))
def test_counted_wait_kernels(asm, kernel):
    src, part, budget, dma, prologue, stores = KERNELS[kernel]
    problems = verify(asm[src], part, budget, dma, prologue, stores)
    assert not problems, "\n".join(problems)


def _steady_wait_line(text, part):
    """Index (in the whole asm text) of the dstr kernel's steady-state counted wait."""
    name, body, _ = isa_guard.kernel_text(text, part)
    start = text.index(name + ":")
    at = text.index("s_waitcnt vmcnt(12)", start)
    return text.index("\n", at) + 1


def test_guard_catches_an_injected_load(asm):
    """A global load the compiler would add inside the counted region (here:
    right after dstr's steady-state wait) is reported."""
    src, part, budget, dma, prologue, stores = KERNELS["dstr"]
    text = asm[src]
    i = _steady_wait_line(text, part)
    bad = text[:i] + "\tglobal_load_dword v0, v[0:1], off\n" + text[i:]
    problems = verify(bad, part, budget, dma, prologue, stores)
    assert any("other load" in p for p in problems), problems


def test_guard_catches_a_dropped_dma(asm):
    """One DMA fewer per step (a wait that would then cover the wrong step)
    is reported."""
    src, part, budget, dma, prologue, stores = KERNELS["dstr"]
    text = asm[src]
    i = _steady_wait_line(text, part)
    j = text.index("global_load_lds_dwordx4", i)
    line_start = text.rindex("\n", 0, j) + 1
    line_end = text.index("\n", j) + 1
    bad = text[:line_start] + text[line_end:]
    problems = verify(bad, part, budget, dma, prologue, stores)
    assert any("DMA between counted waits" in p for p in problems), problems
