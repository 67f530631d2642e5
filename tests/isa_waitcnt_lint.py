"""Lint the gfx950 ISA of a kernel for LDS-DMA pieces that a hand-counted wait leaves in flight.

An LDS-DMA (``buffer_load_* ... lds``) writes LDS with no register destination: nothing orders a ``ds_read`` behind it
except the issuing wave's ``s_waitcnt vmcnt(N)`` followed by a barrier the reader has passed (MI355X_MICROARCH.md item 7;
cdna_hip_programming.md "Read a staged buffer one phase AFTER the wait that retires it").  The kernels here count those
waits by hand (inline asm, each followed by a workgroup barrier), so a wait whose N leaves the piece in flight --
because a path issues fewer vector-memory operations after it than the count assumes (a conditional store or load, a
store the compiler proved dead and deleted, a compiler spill placed elsewhere) -- races its readers silently.

Each LDS-DMA carries its *lag* in its asm text (``; dma-lag K``, default 1): it must be retired by the K-th hand-written
``s_waitcnt vmcnt`` (an inline-asm one) that follows its issue; its readers read after the barrier behind that wait.
The lint runs a monotone dataflow over the kernel's control-flow graph (the structurised ``Flow`` blocks' known scalar
masks resolved as in isa_mfma_lint.py): per program point, each outstanding DMA (instruction, hand waits passed) with the
FEWEST vector-memory operations issued after it on any path reaching that point.  Loads, stores, scratch spills and
LDS-DMA count together, in issue order; every ``s_waitcnt vmcnt(N)`` -- hand-written or compiler-inserted -- retires
the operations with at least N younger ones; at most 63 are outstanding.  A DMA still outstanding at its K-th hand wait
on some path is reported.

usage: python -m tests.isa_waitcnt_lint <file.s> [kernel-symbol] [--lag=K (lag of unannotated DMAs)]   exit 1 on a race
"""
import functools
import heapq
import re
import sys

from tests.isa_mfma_lint import BRANCH_C, parse, sregs

VMEM = ("buffer_", "global_", "scratch_", "flat_")
MAXQ = 63          # the vmcnt counter's capacity: a wave never has more vector-memory operations outstanding
MAX_KEYS = 160     # path distinctions (scalar values, facts) kept per block; beyond, states merge into TOP
INT_EXACT = 4      # loop counters are tracked exactly up to this value, then as ">= INT_EXACT" (so the walk terminates)
MAX_FACTS = 6      # path facts kept (the most recent branch decisions: the structurised re-tests are close by)
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


# ---- scalar path conditions.  A value is True / False (a known 64-bit mask: nonzero / zero), a predicate
# (relation, type, A, B, polarity) from an s_cmp, or absent (unknown).  A branch on a known value takes one successor;
# a branch on a predicate records it as a fact on each successor, so a later test of the same comparison (hipcc
# re-tests `T < ntiles` at every `if` rather than keeping the mask) takes the same side.  Writes to an operand drop the
# facts and values that mention it.
_NEG = {"lt": "ge", "ge": "lt", "gt": "le", "le": "gt", "eq": "lg", "lg": "eq"}
_NO_SDST = ("s_cmp", "s_bitcmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_endpgm", "s_setprio", "s_sleep",
            "s_sethalt", "s_store", "s_dcache", "s_trap", "s_memtime", "s_memrealtime", "s_icache", "s_sendmsg")
_KEEP_SCC = ("s_mov", "s_cselect", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop", "s_load", "s_buffer_load",
             "s_setprio", "s_sleep", "s_memtime", "s_memrealtime", "s_movk", "s_getpc", "s_setpc", "s_swappc")


def _neg(v):
    if v is True or v is False:
        return not v
    if v[0] == "reg":
        return ("reg", v[1], not v[2])
    rel, ty, a, b, pol = v
    return (rel, ty, a, b, not pol)


def _fact_key(v):
    """(fact key, polarity) of a predicate or register-alias value."""
    if v[0] == "reg":
        return ("reg", v[1]), v[2]
    return v[:4], v[4]


def _ival(tok, env):
    """(lo, hi) bounds of an integer operand (hi None: unbounded): a literal, or a 32-bit sgpr set on this path by an
    s_mov of a literal / another tracked sgpr, or by an s_add of a positive literal to one (a loop counter: exact up to
    INT_EXACT, then bounded below by it, so a counter tested against a small constant stays decided)."""
    try:
        v = int(tok, 0)
        return (v, v)
    except ValueError:
        v = env.get(_reg_key(tok))
        return (v[1], v[2]) if isinstance(v, tuple) and v[0] == "int" else None


def _cmp_value(op, toks, env=None):
    m = re.fullmatch(r"s_cmpk?_(eq|lg|lt|le|gt|ge)_(i32|u32|u64)", op)
    if not m or len(toks) < 2:
        return None
    rel, ty = m.groups()
    if env is not None and ty != "u64":
        ia, ib = _ival(toks[0], env), _ival(toks[1], env)
        if ia is not None and ib is not None and min(ia[0], ib[0]) >= 0 and max(ia[0], ib[0]) < (1 << 31):
            (alo, ahi), (blo, bhi) = ia, ib  # non-negative 31-bit bounds: signed and unsigned agree
            inf = float("inf")
            ahi, bhi = (inf if ahi is None else ahi), (inf if bhi is None else bhi)
            lt = True if ahi < blo else (False if alo >= bhi else None)
            le = True if ahi <= blo else (False if alo > bhi else None)
            eq = True if alo == ahi == blo == bhi else (False if ahi < blo or bhi < alo else None)
            r = {"lt": lt, "le": le, "eq": eq, "gt": None if le is None else not le, "ge": None if lt is None else not lt,
                 "lg": None if eq is None else not eq}[rel]
            if r is not None:
                return r
    if rel in ("ge", "gt", "lg"):
        return (_NEG[rel], ty, toks[0], toks[1], False)
    return (rel, ty, toks[0], toks[1], True)


@functools.lru_cache(maxsize=None)
def _reg_key(tok):
    if tok in ("vcc", "exec", "m0", "scc"):
        return tok
    return sregs(tok)


def _overlap(k, reg):
    if isinstance(k, str) or isinstance(reg, str):
        return k == reg
    return k[0] <= reg[1] and reg[0] <= k[1]


def _vgprs(tok):
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return (int(m.group(1)), int(m.group(1)))
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    return (int(m.group(1)), int(m.group(2))) if m else None


def _kill_vgpr(env, rng):
    """A VGPR write: forget the values its lanes held (v_writelane copies of tracked sgprs: hipcc spills loop-carried
    scalars -- a counter, a first-item flag, a mask -- to VGPR lanes and reads them back before each test) and the
    uniform 0 / 1 it held (v_cndmask of a mask: hipcc round-trips some uniform bools through a VGPR)."""
    for k in [k for k in env if isinstance(k, tuple) and k[0] in ("lane", "vval") and rng[0] <= k[1] <= rng[1]]:
        del env[k]


def _mentions(v, reg):
    """Whether value v (a predicate, or a register alias) reads register reg (an sgpr range or a special name)."""
    if not isinstance(v, tuple) or v[0] == "int":
        return False
    if v[0] == "reg":
        return _overlap(v[1], reg)
    for t in (v[2], v[3]):
        k = _reg_key(t)
        if k is None:
            continue
        if isinstance(k, str) or isinstance(reg, str):
            if k == reg:
                return True
        elif k[0] <= reg[1] and reg[0] <= k[1]:
            return True
    return False


def _written(op, toks):
    if op.startswith("s_") and not op.startswith(_NO_SDST) and toks:
        return _reg_key(toks[0])
    if (op.startswith(("v_cmp", "v_readfirstlane", "v_readlane")) or "_co_" in op or op.startswith("v_div_scale")) and toks:
        return _reg_key(toks[0])
    return None


def _kill(env, facts, reg):
    """An sgpr (range) or special register is written: drop what was known about it and the values and facts that read
    it."""
    def hit(k):
        if k == reg:
            return True
        if isinstance(reg, str) or not isinstance(k, tuple):
            return False
        if k[0] in ("lane", "vval"):
            return False
        rng = k[1:] if k[0] == "saved" else k
        return rng[0] <= reg[1] and reg[0] <= rng[1]

    for k in [k for k in env if hit(k)]:
        del env[k]
    for k in [k for k, v in env.items() if _mentions(v, reg)]:
        del env[k]
    for f in [f for f in facts if _mentions(f + (True,), reg)]:
        del facts[f]


def _mask(env, key):
    """Value of a 64-bit mask register pair: tracked as a pair, or as two 32-bit halves a v_readlane pair brought back
    (all ones / zero)."""
    v = env.get(key)
    if v is not None or not isinstance(key, tuple) or key[1] != key[0] + 1:
        return v
    lo, hi = env.get((key[0], key[0])), env.get((key[1], key[1]))
    if lo == hi and lo in (("int", -1, -1), ("int", 0, 0)):
        return lo[1] == -1
    return None


def _known(v, facts):
    """True / False if value v is decided on this path, else None."""
    if v is True or v is False:
        return v
    if isinstance(v, tuple):
        fk, pol = _fact_key(v)
        t = facts.get(fk)
        if t is not None:
            return t == pol
    return None


def transfer(block, state, lag, report):
    """state = (outstanding LDS-DMA {(line, hand waits passed since issue): fewest vector-memory operations issued after
    it on any path reaching here}, scalar values, path facts).  Returns the out-state and the final branch's condition
    (a value, or None), with its sense: the taken successor is reached when the condition is True."""
    q, env, facts = dict(state[0]), dict(state[1]), dict(state[2])
    cond = None
    for ln, raw, op, toks, in_asm in block["ins"]:
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", " ".join(toks))
            if m:
                n = int(m.group(1))
                q = {k: p for k, p in q.items() if p < n}
                if in_asm:  # a hand-counted wait: every DMA still outstanding has passed one more
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
        if in_asm:
            continue
        # scalar values and path facts
        if op.startswith(("s_cbranch_scc", "s_cbranch_vcc")):
            v = env.get("scc" if "scc" in op else "vcc")
            if v is not None:
                cond = v if op in ("s_cbranch_scc1", "s_cbranch_vccnz") else _neg(v)
            continue
        if op.startswith("s_cbranch_exec"):
            if env.get("exec") is True:  # every lane active: execnz always taken, execz never
                cond = op == "s_cbranch_execnz"
            continue
        # exec: known full at entry and after the structurised region that saved it full is closed again
        if "saveexec" in op and toks:
            full = env.get("exec")
            _kill(env, facts, _reg_key(toks[0]))
            env.pop("exec", None)
            sk = _reg_key(toks[0])
            if full is True and isinstance(sk, tuple):
                env[("saved",) + sk] = True
            env.pop("scc", None)
            continue
        if toks and toks[0] == "exec":
            src = _reg_key(toks[2]) if op == "s_or_b64" and len(toks) == 3 and toks[1] == "exec" else None
            restored = src is not None and not isinstance(src, str) and env.get(("saved",) + tuple(src)) is True
            env.pop("exec", None)
            if restored:
                env["exec"] = True
            env.pop("scc", None)
            continue
        if op.startswith("v_readlane_b32") and len(toks) == 3:
            sk = _reg_key(toks[0])
            vr = _vgprs(toks[1])
            val = env.get(("lane", vr[0], toks[2])) if vr else None
            if isinstance(sk, tuple):
                _kill(env, facts, sk)
                if val is not None:
                    env[sk] = val
            continue
        if op.startswith("v_writelane_b32") and len(toks) == 3 and _vgprs(toks[0]):
            val = env.get(_reg_key(toks[1]))
            lk = ("lane", _vgprs(toks[0])[0], toks[2])
            if isinstance(val, tuple) and val[0] == "int":
                env[lk] = val
            else:
                env.pop(lk, None)
            continue
        if toks and (op.startswith("v_") or op.startswith(("ds_read", "ds_load"))) and _vgprs(toks[0]) is not None:
            _kill_vgpr(env, _vgprs(toks[0]))
            if (op.startswith("v_cndmask_b32") and len(toks) == 4 and toks[1:3] == ["0", "1"] and env.get("exec") is True
                    and _vgprs(toks[0])[0] == _vgprs(toks[0])[1]):
                mv = _mask(env, _reg_key(toks[3]))
                if mv is not None:
                    env[("vval", _vgprs(toks[0])[0])] = mv  # every lane: 1 where the mask is set (a uniform mask)
                continue
        if (re.fullmatch(r"v_cmp_(ne|eq)_u32_e64", op) and len(toks) == 3 and env.get("exec") is True
                and isinstance(_reg_key(toks[0]), tuple)):
            vr = _vgprs(toks[2]) if toks[1] in ("0", "1") else (_vgprs(toks[1]) if toks[2] in ("0", "1") else None)
            lit = toks[1] if toks[1] in ("0", "1") else toks[2]
            mv = env.get(("vval", vr[0])) if vr else None
            w = _reg_key(toks[0])
            _kill(env, facts, w)
            if mv is not None:  # (v == 1) is the mask, (v == 0) its negation
                env[w] = mv if (op.startswith("v_cmp_eq") == (lit == "1")) else _neg(mv)
            continue
        newv = None
        cv = _cmp_value(op, toks, env)
        if op.startswith("s_cselect_b64") and len(toks) == 3 and toks[1:] in (["-1", "0"], ["0", "-1"]):
            sv = env.get("scc")
            newv = None if sv is None else (sv if toks[1] == "-1" else _neg(sv))
        elif op == "s_mov_b64" and len(toks) == 2 and toks[1] in ("0", "-1"):
            newv = toks[1] == "-1"
        elif op == "s_mov_b64" and len(toks) == 2 and _mask(env, _reg_key(toks[1])) is not None:
            newv = _mask(env, _reg_key(toks[1]))
        elif op in ("s_xor_b64", "s_not_b64") and len(toks) >= 2 and (op == "s_not_b64" or "-1" in toks[1:]):
            src = [t for t in toks[1:] if t != "-1"]
            sv = _mask(env, _reg_key(src[0])) if src else None
            newv = None if sv is None else _neg(sv)
        elif op in ("s_mov_b32", "s_movk_i32") and len(toks) == 2 and _ival(toks[1], env) is not None:
            newv = ("int",) + _ival(toks[1], env)
        elif op in ("s_add_i32", "s_add_u32") and len(toks) == 3:
            ia, ib = _ival(toks[1], env), _ival(toks[2], env)
            if ia is not None and ib is not None and ia[0] == ia[1] and ib[0] != ib[1]:
                ia, ib = ib, ia  # the literal / exact operand second
            if ia is not None and ib is not None and ib[0] == ib[1]:
                lo, hi = ia[0] + ib[0], (None if ia[1] is None else ia[1] + ib[0])
                newv = ("int", lo, hi) if lo <= INT_EXACT or ib[0] <= 0 else ("int", INT_EXACT, None)
        elif op in ("s_and_b64", "s_or_b64", "s_andn2_b64") and len(toks) == 3 and "exec" not in toks[1:]:
            va, vb = (_mask(env, _reg_key(t)) if t not in ("0", "-1") else t == "-1" for t in toks[1:])
            if op == "s_andn2_b64" and vb is not None:
                vb = _neg(vb)
            if op == "s_or_b64":
                newv = True if True in (va, vb) else (vb if va is False else (va if vb is False else None))
            else:
                newv = False if False in (va, vb) else (vb if va is True else (va if vb is True else None))
        elif op in ("s_and_b64", "s_andn2_b64") and len(toks) == 3 and toks[1] == "exec":
            rk = _reg_key(toks[2])
            sv = _mask(env, rk)  # exec is non-zero in any block a wave executes
            if sv is None and rk is not None and not isinstance(rk, str):
                kn = facts.get(("reg", rk))
                sv = kn if kn is not None else ("reg", rk, True)  # unknown mask: the branch on it decides it
            newv = None if sv is None else (sv if op == "s_and_b64" else _neg(sv))
        w = _written(op, toks)
        if w is not None:
            _kill(env, facts, w)
            if newv is not None:
                env[w] = newv
                if isinstance(newv, bool) and isinstance(w, tuple) and w[1] == w[0] + 1:  # a constant mask: its halves too
                    env[(w[0], w[0])] = env[(w[1], w[1])] = ("int", -1 if newv else 0, -1 if newv else 0)
        if cv is not None:
            env["scc"] = cv  # (a bool when both operands are known)
        elif op in ("s_and_b64", "s_andn2_b64") and w == "vcc" and newv is not None:
            env["scc"] = newv  # scc = (result != 0)
        elif not op.startswith(_KEEP_SCC) and (op.startswith("s_") or "_co_" in op):
            env.pop("scc", None)
    return (q, env, facts), cond


def lint(lines, default_lag=1):
    """-> races [(wait line, DMA line, hand waits passed)]: the DMA may still be in flight at the hand-written wait that
    must retire it.  Monotone dataflow over the CFG: per block and (scalar values, path facts), the outstanding DMAs
    with the fewest operations issued after them over all paths (a join of min), iterated to the fixed point."""
    lag = annotate(lines, default_lag)
    blocks = parse(lines)
    index = {b["label"]: k for k, b in enumerate(blocks) if b["label"]}

    def succs(k, cond, facts):
        """[(successor, facts on that edge)]"""
        b = blocks[k]
        tgt = [index[t] for t in b["succ"] if t in index]
        last = b["ins"][-1][2] if b["ins"] else ""
        nxt = [k + 1] if b["fall"] and k + 1 < len(blocks) else []
        if last in BRANCH_C and last.startswith(("s_cbranch_scc", "s_cbranch_vcc", "s_cbranch_exec")) and cond is not None:
            kn = _known(cond, facts)
            if kn is True:
                return [(t, facts) for t in tgt]
            if kn is False:
                return [(t, facts) for t in nxt]
            ft, ff = dict(facts), dict(facts)
            if isinstance(cond, tuple):
                fk, pol = _fact_key(cond)
                for f_, v_ in ((ft, pol), (ff, not pol)):
                    f_.pop(fk, None)
                    f_[fk] = v_  # most recent last
                    while len(f_) > MAX_FACTS:  # forget the oldest (sound: fewer facts = more paths)
                        del f_[next(iter(f_))]
            return [(t, ft) for t in tgt] + [(t, ff) for t in nxt]
        return [(t, facts) for t in tgt + nxt]

    def key_of(env, facts):
        return (frozenset(env.items()), tuple(facts.items()))

    state_in = [dict() for _ in blocks]  # block -> {(scalar values, facts): {dma key: min ops after}}
    k0 = key_of({"exec": True}, {})
    state_in[0][k0] = {}
    work = [(0, 0, k0)]  # (block, tie-breaker, key): blocks in layout order converge in few passes
    queued = {(0, k0)}
    tick = 0
    while work:
        k, _t, key = heapq.heappop(work)
        queued.discard((k, key))
        out, cond = transfer(blocks[k], (state_in[k][key], dict(key[0]), dict(key[1])), lag, None)
        for s_, facts in succs(k, cond, out[2]):
            nkey = key_of(out[1], facts)
            if nkey not in state_in[s_] and len(state_in[s_]) >= MAX_KEYS:
                # too many path distinctions here: merge into a state that keeps only what it knows about exec (full, and
                # the masks the open structurised regions saved)
                kept = {kk: v for kk, v in out[1].items() if kk == "exec" or (isinstance(kk, tuple) and kk[0] == "saved")}
                nkey = key_of(kept, {})
            cur = state_in[s_].get(nkey)
            if cur is None:
                state_in[s_][nkey] = dict(out[0])
                if (s_, nkey) not in queued:
                    queued.add((s_, nkey))
                    tick += 1
                    heapq.heappush(work, (s_, tick, nkey))
                continue
            changed = False
            for d, p in out[0].items():
                if p < cur.get(d, MAXQ):
                    cur[d] = p
                    changed = True
            if changed and (s_, nkey) not in queued:
                queued.add((s_, nkey))
                tick += 1
                heapq.heappush(work, (s_, tick, nkey))
    report = []
    for k, b in enumerate(blocks):
        for key, q in state_in[k].items():
            transfer(b, (q, dict(key[0]), dict(key[1])), lag, report)
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
            print(f"  hand wait at line {bl}: LDS-DMA of line {dl} still in flight (hand wait {b} after its issue)")
        rc |= 1 if races else 0
    return rc


if __name__ == "__main__":
    sys.exit(main())
