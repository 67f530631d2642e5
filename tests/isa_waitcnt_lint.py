"""Lint the gfx950 ISA of a kernel for LDS-DMA rows that are still in flight when their readers may read them.

An LDS-DMA (``buffer_load_* ... lds``) writes LDS with no register destination: nothing orders a ``ds_read`` behind it
except the issuing wave's ``s_waitcnt vmcnt(N)`` followed by a barrier the reader has passed (MI355X_MICROARCH.md item 7;
cdna_hip_programming.md "Read a staged buffer one phase AFTER the wait that retires it").  The kernels here count those
waits by hand (inline asm), so a wait whose N leaves the piece in flight -- because a path issues fewer vector-memory
operations after it than the count assumes (a conditional store or load, a compiler spill, an operation the compiler
moved) -- races its readers silently.

Each LDS-DMA carries its *lag* in the asm text (``; dma-lag K``, default 1): its data is read after the K-th
``s_barrier`` that follows its issue, by any wave.  The lint walks every control-flow path (the structurised
``Flow`` blocks' known scalar masks resolved as in isa_mfma_lint.py) with the wave's queue of outstanding
vector-memory operations (loads, stores, scratch spills and LDS-DMA count together, in issue order; ``s_waitcnt
vmcnt(N)`` -- hand-written or compiler-inserted -- retires all but the youngest N; at most 63 are outstanding) and
reports every barrier at which a DMA reaches its K-th barrier still outstanding on some path.

usage: python -m tests.isa_waitcnt_lint <file.s> [kernel-symbol] [--lag=K (lag of unannotated DMAs)]   exit 1 on a race
"""
import re
import sys

from tests.isa_mfma_lint import BRANCH_C, BRANCH_U, parse, sregs

VMEM = ("buffer_", "global_", "scratch_", "flat_")
MAXQ = 63          # the vmcnt counter's capacity: a wave never has more vector-memory operations outstanding
_LAG = re.compile(r"dma-lag\s+(\d+)")


def _vmcnt(toks):
    for t in toks:
        m = re.fullmatch(r"vmcnt\((\d+)\)", t.strip())
        if m:
            return int(m.group(1))
    return None


def annotate(lines, default=1):
    """Lag of each LDS-DMA line: the ``dma-lag K`` comment in its asm block (else ``default``)."""
    lag = {}
    cur = None
    for i, raw in enumerate(lines):
        if "ASMSTART" in raw:
            cur = None
        m = _LAG.search(raw)
        if m:
            cur = int(m.group(1))
        s = raw.split(";")[0].strip()
        if s.startswith(("buffer_load", "global_load")) and re.search(r"\blds\b", s):
            lag[i + 1] = cur if cur is not None else default
    # a lag comment may follow the instruction inside the same asm block
    for i, raw in enumerate(lines):
        s = raw.split(";")[0].strip()
        if (i + 1) in lag:
            m = _LAG.search(raw)
            if m:
                lag[i + 1] = int(m.group(1))
    return lag


def transfer(block, state, lag, report):
    """state = (outstanding LDS-DMA {(line, barriers passed since issue): fewest vector-memory operations issued after it
    on any path reaching here}, scalar constants).  A wait vmcnt(N) retires the DMAs with >= N operations after them
    (all operations count, in issue order); an operation at MAXQ or more behind the youngest is retired (the counter's
    capacity).  Returns the out-state and the taken-ness of a final conditional branch on a known constant (see
    isa_mfma_lint.transfer)."""
    q, sc = dict(state[0]), dict(state[1])
    taken = None
    for ln, raw, op, toks, in_asm in block["ins"]:
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", " ".join(toks))
            if m:
                n = int(m.group(1))
                q = {k: p for k, p in q.items() if p < n}
            continue
        if op == "s_barrier":
            nq = {}
            for (dl, b), p in q.items():
                b += 1
                if b >= lag.get(dl, 1) and report is not None:
                    report.append((ln, dl, b))
                key = (dl, min(b, 8))
                nq[key] = min(p, nq.get(key, MAXQ))
            q = nq
            continue
        if op.startswith(VMEM):
            q = {k: p + 1 for k, p in q.items() if p + 1 < MAXQ}
            s = raw.split(";")[0]
            if op.startswith(("buffer_load", "global_load")) and re.search(r"\blds\b", s):
                q[(ln, 0)] = 0
            continue
        # scalar constant tracking for the structurised Flow blocks (as isa_mfma_lint.transfer)
        if op.startswith("s_") and toks:
            dst = "vcc" if toks[0] == "vcc" else sregs(toks[0])
            if op == "s_mov_b64" and dst is not None and len(toks) > 1 and toks[1] in ("0", "-1"):
                sc[dst] = int(toks[1])
            elif op in ("s_andn2_b64", "s_and_b64") and toks[0] == "vcc" and len(toks) > 2 and toks[1] == "exec":
                src = sregs(toks[2])
                v = sc.get(src)
                if v is None:
                    sc.pop("vcc", None)
                else:
                    sc["vcc"] = (v == 0) if op == "s_andn2_b64" else (v != 0)
            elif dst is not None:
                sc.pop(dst, None)
            if op == "s_cbranch_vccnz" and "vcc" in sc:
                taken = bool(sc["vcc"])
            elif op == "s_cbranch_vccz" and "vcc" in sc:
                taken = not sc["vcc"]
        if op.startswith("v_cmp"):
            sc.pop("vcc", None)
    return (q, sc), taken


def lint(lines, default_lag=1):
    """-> races [(barrier line, DMA line, barriers passed)]: the DMA may still be in flight at the barrier after which
    its readers read it.  Monotone dataflow over the CFG: per block and set of known scalar constants, the outstanding
    DMAs with the fewest operations issued after them over all paths (a join of min), iterated to the fixed point."""
    lag = annotate(lines, default_lag)
    blocks = parse(lines)
    index = {b["label"]: k for k, b in enumerate(blocks) if b["label"]}

    def succs(k, taken):
        b = blocks[k]
        tgt = [index[t] for t in b["succ"] if t in index]
        last = b["ins"][-1][2] if b["ins"] else ""
        if last in BRANCH_C and taken is not None:
            return tgt if taken else ([k + 1] if k + 1 < len(blocks) else [])
        out = list(tgt)
        if b["fall"] and k + 1 < len(blocks):
            out.append(k + 1)
        return out

    state_in = [dict() for _ in blocks]  # block -> {frozen scalar constants: {dma key: min ops after}}
    state_in[0][frozenset()] = {}
    work = [(0, frozenset())]
    while work:
        k, key = work.pop()
        out, taken = transfer(blocks[k], (state_in[k][key], dict(key)), lag, None)
        nkey = frozenset(out[1].items())
        for s_ in succs(k, taken):
            cur = state_in[s_].get(nkey)
            if cur is None:
                state_in[s_][nkey] = dict(out[0])
                work.append((s_, nkey))
                continue
            changed = False
            for d, p in out[0].items():
                if p < cur.get(d, MAXQ):
                    cur[d] = p
                    changed = True
            if changed and (s_, nkey) not in work:
                work.append((s_, nkey))
    report = []
    for k, b in enumerate(blocks):
        for key, q in state_in[k].items():
            transfer(b, (q, dict(key)), lag, report)
    return sorted(set(report))


def kernels(asm_text, pattern=r"^(_Z\w*kernel\w*):"):
    lines = asm_text.split("\n")
    out = {}
    for i, l in enumerate(lines):
        m = re.match(pattern, l)
        if m:
            end = next((j for j in range(i + 1, len(lines)) if lines[j].startswith(".Lfunc_end")), len(lines))
            out[m.group(1)] = lines[i:end + 1]
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--lag=")]
    dflt = int(next((a[6:] for a in sys.argv[1:] if a.startswith("--lag=")), "1"))
    path = args[0]
    sym = args[1] if len(args) > 1 else ""
    text = open(path).read()
    ks = kernels(text)
    rc = 0
    for name, lines in ks.items():
        if sym and sym not in name:
            continue
        races = lint(lines, dflt)
        ndma = len(annotate(lines, dflt))
        print(f"{name}: {ndma} LDS-DMA instructions, {len(races)} race(s)")
        for bl, dl, b in races[:20]:
            print(f"  barrier at line {bl}: LDS-DMA of line {dl} still in flight after {b} barrier(s)")
        rc |= 1 if races else 0
    return rc


if __name__ == "__main__":
    sys.exit(main())
