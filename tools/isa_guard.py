"""CPU-side ISA guard for the kernels whose pipelines rest on hand-counted
`s_waitcnt vmcnt(N)` (dstr_kernel, lpd_kernel, lpw_kernel).

The counted waits assume that between two of them a wave issues exactly the
vector-memory instructions the source writes: the step's LDS-DMA
(`global_load_lds_dwordx4`, inline asm) and, on some paths, a chunk's output
stores.  A compiler that adds a VMEM instruction inside that region (a spill,
a scratch access, a hoisted load) changes what the next wait covers, and
only the GPU tests would notice.  This module reads the device assembly that
clang emits for the product sources (no GPU needed) and checks, per kernel:

  * no private segment (scratch), no VGPR spills, VGPRs within the launch
    shape's budget;
  * along every control-flow path from one counted wait (an inline-asm
    `s_waitcnt vmcnt(N)`, N > 0) to the next, the number of DMA, other
    load and store instructions issued, as a data-flow over the kernel's
    basic blocks; a `vmcnt(0)` drain starts the count afresh.

The expectations live in tests/test_isa_guard.py next to the source lines
that fix them.
"""
import re
import subprocess
from collections import defaultdict

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
CAP = 99      # "many": counts above WIDEN jump here, so loops with VMEM reach a fixed point
WIDEN = (None, 24, 4, 12)  # per counter (dma, loads, stores): above it the count becomes CAP
FACT_AGE = 4
MAX_VISITS = 2_000_000
TRACK = (0,)  # counters followed along paths: the DMA (the other VMEM: inventory())


def device_asm(src, out, include_dirs=(), defines=()):
    """clang -S of one .hip file for gfx950 (device code only)."""
    cmd = ["/opt/rocm/lib/llvm/bin/clang++", "-x", "hip", "--offload-arch=gfx950", "-O3", "-std=c++17",
           "-mcode-object-version=5", "--cuda-device-only", "-S", "-o", out, src]
    cmd += [f"-I{d}" for d in include_dirs] + [f"-D{d}" for d in defines]
    subprocess.run(cmd, check=True)
    with open(out) as f:
        return f.read()


def kernel_text(asm, symbol_part):
    """The instruction lines of the one kernel whose mangled name contains
    `symbol_part`, and its metadata block (.amdhsa_kernel ... .end_amdhsa_kernel
    plus the YAML note entries)."""
    m = [x for x in re.finditer(r"^(_Z\S+):", asm, re.M) if symbol_part in x.group(1)]
    if len(m) != 1:
        raise KeyError(f"{symbol_part}: {len(m)} kernels match")
    name = m[0].group(1)
    start = m[0].end()
    end = asm.index(".Lfunc_end", start)
    body = asm[start:end]
    meta = {}
    k = asm.index(f".amdhsa_kernel {name}")
    for line in asm[k:asm.index(".end_amdhsa_kernel", k)].splitlines():
        p = line.split()
        if len(p) == 2 and p[0].startswith(".amdhsa_"):
            meta[p[0]] = int(p[1]) if p[1].lstrip("-").isdigit() else p[1]
    # the code-object note: .vgpr_count, .vgpr_spill_count, .private_segment_fixed_size
    # (the keys after the kernel's .name, up to its .wavefront_size)
    note = asm.index(f".name:           {name}")
    blk = asm[note:asm.index(".wavefront_size", note)]
    for key in ("private_segment_fixed_size", "vgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                "sgpr_count", "uses_dynamic_stack"):
        mm = re.search(rf"\.{key}:\s+(\w+)", blk)
        if mm:
            v = mm.group(1)
            meta[key] = int(v) if v.isdigit() else v
    return name, body, meta


def blocks_of(body):
    """Basic blocks: {label, ins, succ}.  An instruction is a dict with `op`,
    `text` and `asm` (inside ;;#ASMSTART / ;;#ASMEND).  A block ends at a
    label, after a branch or after s_endpgm; successors are the branch
    targets plus the next block unless the block ends unconditionally."""
    blocks = [{"label": "<entry>", "ins": [], "targets": [], "term": None}]
    in_asm = False
    for raw in body.splitlines():
        s = raw.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        m = re.match(r"^(\.LBB\d+_\d+):", raw)
        if m:
            blocks.append({"label": m.group(1), "ins": [], "targets": [], "term": None})
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        text = s.split(";")[0].strip()
        if not text:
            continue
        op = text.split()[0]
        b = blocks[-1]
        b["ins"].append({"op": op, "text": text, "asm": in_asm})
        if op == "s_branch" or op.startswith("s_cbranch_") or op in ("s_endpgm", "s_setpc_b64"):
            b["term"] = "cbr" if op.startswith("s_cbranch_") else "end" if op in ("s_endpgm", "s_setpc_b64") else "br"
            if op != "s_endpgm" and op != "s_setpc_b64":
                b["targets"] = [text.split()[1]]
            blocks.append({"label": f"<after-{len(blocks)}>", "ins": [], "targets": [], "term": None})
    for i, b in enumerate(blocks):
        fall = b["term"] in (None, "cbr") and i + 1 < len(blocks)
        b["succ"] = b["targets"] + ([blocks[i + 1]["label"]] if fall else [])
    return blocks


def vmcnt_of(text):
    m = re.search(r"vmcnt\((\d+)\)", text)
    return int(m.group(1)) if m else None


def classify(op):
    if op.startswith("global_load_lds") or op.startswith("buffer_load_lds"):
        return 0  # DMA into LDS
    if "store" in op or "atomic" in op:
        return 2
    return 1      # any other load


def sregs(tok):
    """SGPR indices named by an operand token (s7, s[6:7]); 'vcc' for vcc."""
    tok = tok.rstrip(",")
    if tok in ("vcc", "vcc_lo", "vcc_hi"):
        return {"vcc"}
    m = re.fullmatch(r"s(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


NO_DEST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_barrier", "s_endpgm",
           "s_sleep", "s_setprio", "s_dcache", "s_sendmsg", "s_trap", "s_icache", "buffer_", "global_",
           "ds_", "flat_", "scratch_", "s_store", "s_buffer_store", "s_atomic")


def step_known(known, ins):
    """Transfer of the branch-flag facts across one instruction.  `known`:
    frozenset of (reg, value, age): SGPR pairs set to -1 / 0 by s_mov_b64
    (the structurizer's flags) and ("vcc", "z" | "nz", age)."""
    op, text = ins["op"], ins["text"]
    toks = text.split()[1:]
    k = {r: (v, a) for r, v, a in known}
    if "saveexec" in op or op.startswith("v_cmpx") or (toks and toks[0].rstrip(",") == "exec"):
        # exec: nonzero at entry; a restore (s_or_b64 exec, exec, saved /
        # s_mov_b64 exec, saved) makes it nonzero again, any other write may
        # leave it empty (a divergent region)
        restore = op in ("s_or_b64", "s_mov_b64") and toks and toks[0].rstrip(",") == "exec" and \
            (op == "s_mov_b64" or toks[1].rstrip(",") == "exec")
        k.pop("exec", None)
        if restore:
            k["exec"] = ("nz", 0)
        return frozenset((r, v, a) for r, (v, a) in k.items())
    if (op.startswith("v_cmp") and "_e32" in op) or op.startswith("v_cmpx"):
        if "vcc" not in k:
            return known
        k.pop("vcc")
        return frozenset((r, v, a) for r, (v, a) in k.items())
    if not toks or op.startswith(NO_DEST):
        return known
    dst = sregs(toks[0])
    if not dst:
        return known
    hit = [r for r in k if (r == "vcc" and "vcc" in dst) or (r not in ("vcc", "exec") and set(r) & dst)]
    for r in hit:
        del k[r]
    if op == "s_mov_b64" and len(toks) == 2 and toks[1] in ("-1", "0") and "vcc" not in dst:
        k[tuple(sorted(dst))] = (int(toks[1]), 0)
    elif dst == {"vcc"} and op in ("s_andn2_b64", "s_and_b64") and len(toks) == 3 and toks[1].rstrip(",") == "exec":
        r = tuple(sorted(sregs(toks[2])))
        if r in k:
            zero = (k[r][0] == -1) if op == "s_andn2_b64" else (k[r][0] == 0)
            k["vcc"] = ("z" if zero else "nz", 0)
    elif not hit:
        return known
    return frozenset((r, v, a) for r, (v, a) in k.items())


def analyze(body):
    """Abstract interpretation over the kernel's basic blocks.  A state is
    (origin, dma, loads, stores, flags): the VMEM instructions issued since
    the last counted wait (origin "W"), drain ("Z", a vmcnt(0)) or kernel
    entry ("E"), and the structurizer's branch flags, so that an if / else
    pair compiled as two guarded blocks counts one arm, not zero or two.
    Returns (waits, scratch_ops): waits = [(block, index, N, states)] for
    every counted wait (inline-asm vmcnt(N), N > 0)."""
    blocks = blocks_of(body)
    idx = {b["label"]: i for i, b in enumerate(blocks)}
    IN = defaultdict(set)
    IN[0].add(("E", 0, 0, 0, frozenset({("exec", "nz", 0)})))
    waits = {}
    scratch = []
    work = [0]
    visits = 0
    while work:
        visits += 1
        if visits > MAX_VISITS:
            raise RuntimeError("isa_guard: no fixed point (state explosion)")
        bi = work.pop()
        b = blocks[bi]
        st = set(IN[bi])
        for k, ins in enumerate(b["ins"]):
            op, text = ins["op"], ins["text"]
            if op.startswith("scratch_"):
                scratch.append(text)
            if op == "s_waitcnt":
                n = vmcnt_of(text)
                if n == 0:
                    st = {("Z", 0, 0, 0, x[4]) for x in st}
                elif n is not None and ins["asm"]:
                    key = (bi, k)
                    prev = waits.get(key, (n, set()))[1]
                    waits[key] = (n, prev | {x[:4] for x in st})
                    st = {("W", 0, 0, 0, x[4]) for x in st}
                continue
            if VMEM.match(op) and classify(op) in TRACK:
                c = classify(op) + 1
                st = {tuple(v if i != c else (v + 1 if v < WIDEN[c] else CAP) for i, v in enumerate(x)) for x in st}
            st = {x[:4] + (step_known(x[4], ins),) for x in st}
        last = b["ins"][-1] if b["ins"] else None
        for x in st:
            succ = list(b["succ"])
            # facts age at the block boundary; old ones are dropped
            aged = frozenset((r, v, a if r == "exec" else a + 1) for r, v, a in x[4]
                             if r == "exec" or a + 1 <= FACT_AGE)
            if last and last["op"] in ("s_cbranch_vccnz", "s_cbranch_vccz", "s_cbranch_execnz",
                                       "s_cbranch_execz") and b["targets"]:
                reg = "exec" if "exec" in last["op"] else "vcc"
                v = {r: vv for r, vv, _ in x[4]}.get(reg)
                taken = None if v is None else (v == "nz") == last["op"].endswith("nz")
                if taken is True:
                    succ = b["targets"]
                elif taken is False:
                    succ = [s_ for s_ in succ if s_ not in b["targets"]]
            y = x[:4] + (aged,)
            for lab in succ:
                j = idx.get(lab)
                if j is not None and y not in IN[j]:
                    IN[j].add(y)
                    work.append(j)
    out = [(blocks[bi]["label"], k, n, sorted(s)) for (bi, k), (n, s) in sorted(waits.items())]
    return out, scratch


def loops(blocks):
    """Natural loops of the CFG: {header index: set of block indices}, from
    the back edges (u -> h with h dominating u)."""
    n = len(blocks)
    idx = {b["label"]: i for i, b in enumerate(blocks)}
    succ = [[idx[l] for l in b["succ"] if l in idx] for b in blocks]
    pred = [[] for _ in range(n)]
    for u in range(n):
        for v in succ[u]:
            pred[v].append(u)
    reach = {0}
    stack = [0]
    while stack:
        u = stack.pop()
        for v in succ[u]:
            if v not in reach:
                reach.add(v)
                stack.append(v)
    dom = [set(reach) for _ in range(n)]
    dom[0] = {0}
    changed = True
    while changed:
        changed = False
        for v in sorted(reach):
            if v == 0:
                continue
            ps = [dom[u] for u in pred[v] if u in reach]
            d = set.intersection(*ps) | {v} if ps else {v}
            if d != dom[v]:
                dom[v] = d
                changed = True
    out = defaultdict(set)
    for u in reach:
        for h in succ[u]:
            if h in dom[u]:  # back edge u -> h
                body = {h, u}
                stack = [u]
                while stack:
                    x = stack.pop()
                    for p_ in pred[x]:
                        if p_ not in body and p_ in reach:
                            body.add(p_)
                            stack.append(p_)
                out[h] |= body
    return dict(out)


def loop_segments(body):
    """Per counted wait, the (dma, loads, stores) issued along the paths that
    stay inside the innermost natural loop holding it, from that wait to the
    next counted one: the steady state of the loop.  A drain (vmcnt(0)) ends a
    path.  Returns [(N, block label, sorted set of (dma, loads, stores))]."""
    blocks = blocks_of(body)
    idx = {b["label"]: i for i, b in enumerate(blocks)}
    lp = loops(blocks)
    res = []
    for bi, b in enumerate(blocks):
        for k, ins in enumerate(b["ins"]):
            if not (ins["op"] == "s_waitcnt" and ins["asm"] and (vmcnt_of(ins["text"]) or 0) > 0):
                continue
            inner = min((body_ for body_ in lp.values() if bi in body_), key=len, default=None)
            if inner is None:
                continue
            counts = set()
            seen = set()
            work = [(bi, k + 1, (0, 0, 0), frozenset({("exec", "nz", 0)}))]
            while work:
                item = work.pop()
                if item in seen:
                    continue
                seen.add(item)
                cb, ck, cnt, facts = item
                blk = blocks[cb]
                stop = False
                for ins2 in blk["ins"][ck:]:
                    op = ins2["op"]
                    if op == "s_waitcnt" and vmcnt_of(ins2["text"]) is not None:
                        n2 = vmcnt_of(ins2["text"])
                        if n2 == 0:
                            stop = True          # a drain: the path leaves the counted regime
                            break
                        if ins2["asm"]:
                            counts.add(cnt)
                            stop = True
                            break
                    if VMEM.match(op):
                        c = classify(op)
                        cnt = tuple(min(v + 1, CAP) if i == c else v for i, v in enumerate(cnt))
                    facts = step_known(facts, ins2)
                if stop or max(cnt) >= CAP:   # a capped path is a per-packet store loop: no wait ahead
                    continue
                last = blk["ins"][-1] if blk["ins"] else None
                succ = list(blk["succ"])
                if last and last["op"] in ("s_cbranch_vccnz", "s_cbranch_vccz", "s_cbranch_execnz",
                                           "s_cbranch_execz") and blk["targets"]:
                    reg = "exec" if "exec" in last["op"] else "vcc"
                    v = {r: vv for r, vv, _ in facts}.get(reg)
                    taken = None if v is None else (v == "nz") == last["op"].endswith("nz")
                    if taken is True:
                        succ = blk["targets"]
                    elif taken is False:
                        succ = [x for x in succ if x not in blk["targets"]]
                aged = frozenset((r, v, a if r == "exec" else a + 1) for r, v, a in facts
                                 if r == "exec" or a + 1 <= FACT_AGE)
                for lab in succ:
                    j = idx.get(lab)
                    if j is not None and j in inner:
                        work.append((j, 0, cnt, aged))
            res.append((vmcnt_of(ins["text"]), b["label"], sorted(counts)))
    return res


def check(asm, part):
    """(metadata, steady segments, entry DMA counts) of one kernel: the facts
    tests/test_isa_guard.py asserts."""
    name, body, meta = kernel_text(asm, part)
    waits, scratch = analyze(body)
    entry = sorted({x[1] for _, _, _, st in waits for x in st if x[0] == "E"})
    return {"name": name, "meta": meta, "scratch_ops": len(scratch), "steady": loop_segments(body),
            "entry_dma": entry}


def summary(body):
    """{N: sorted set of (origin, dma, loads, stores)} over the counted waits."""
    waits, scratch = analyze(body)
    res = defaultdict(set)
    for _, _, n, s in waits:
        res[n] |= set(s)
    return {n: sorted(v) for n, v in res.items()}, scratch


if __name__ == "__main__":
    import sys
    asm = open(sys.argv[1]).read()
    for part in sys.argv[2:]:
        name, body, meta = kernel_text(asm, part)
        s, scr = summary(body)
        print(name, {k: meta.get(k) for k in ("vgpr_count", "vgpr_spill_count", "private_segment_fixed_size",
                                              "sgpr_spill_count")})
        for n, v in sorted(s.items()):
            print(f"  vmcnt({n}): {v}")
        print("  scratch ops:", len(scr))
        for n, lab, c in loop_segments(body):
            print(f"  steady vmcnt({n}) at {lab}: (dma, loads, stores) between waits {c}")
