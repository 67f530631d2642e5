"""Lint the gfx950 ISA of a kernel for touches of an inline-asm MFMA's result before its hazard pad.

hipcc cannot see MFMAs issued from inline asm (csrc/mfma_agpr.h), so it inserts no wait states between such an MFMA
and a later VALU / DS / VMEM instruction that reads, overwrites or copies (v_accvgpr_*) its destination registers.
The kernels pad with pad_mfma() (s_nop 7; s_nop 7; s_nop 3 inside asm) before the accumulators are touched; this
checks, over the control-flow graph of the kernel, that nothing but further asm blocks (dependent MFMAs need no wait
states) touches an asm-MFMA destination on any path between the MFMA and such a pad.

usage: python tools/isa_mfma_lint.py <file.s> [kernel-symbol]      exit 1 if a hazard is found
"""
import re
import sys

BRANCH_U = ("s_branch",)
BRANCH_C = ("s_cbranch_scc0", "s_cbranch_scc1", "s_cbranch_vccz", "s_cbranch_vccnz", "s_cbranch_execz", "s_cbranch_execnz")


def vregs(tok):
    """Vector registers of an operand: VGPR n -> n, AGPR n -> 1000 + n (an asm MFMA may accumulate in either half)."""
    m = re.fullmatch(r"([va])(\d+)", tok)
    if m:
        return {int(m.group(2)) + (1000 if m.group(1) == "a" else 0)}
    m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        base = 1000 if m.group(1) == "a" else 0
        return set(range(int(m.group(2)) + base, int(m.group(3)) + base + 1))
    return set()


def parse(lines):
    """-> list of blocks: (label, [(lineno, raw, op, toks, in_asm)], successors labels/None for fallthrough)."""
    blocks = []
    cur = {"label": None, "ins": [], "succ": [], "fall": True}
    in_asm = False
    for i, raw in enumerate(lines):
        s = raw.split(";")[0].strip()
        if "ASMSTART" in raw:
            in_asm = True
            continue
        if "ASMEND" in raw:
            in_asm = False
            continue
        if not s:
            continue
        if s.endswith(":"):
            blocks.append(cur)
            cur = {"label": s[:-1], "ins": [], "succ": [], "fall": True}
            continue
        if s.startswith("."):
            continue
        op, _, rest = s.partition(" ")
        toks = [t.strip() for t in rest.split(",")] if rest else []
        cur["ins"].append((i + 1, raw.strip(), op, toks, in_asm))
        if op in BRANCH_U or op in BRANCH_C or op == "s_endpgm":
            if op in BRANCH_U or op in BRANCH_C:
                cur["succ"].append(toks[0])
            cur["fall"] = op in BRANCH_C
            blocks.append(cur)
            cur = {"label": None, "ins": [], "succ": [], "fall": True}
    blocks.append(cur)
    return [b for b in blocks if b["ins"] or b["label"]]


def sregs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return (int(m.group(1)), int(m.group(2)))
    m = re.fullmatch(r"s(\d+)", tok)
    return (int(m.group(1)), int(m.group(1))) if m else None


def transfer(block, state, report):
    """state = (pending {vgpr: line}, scalar constants {sgpr range: 0 / -1 / 'vcc'}).  Returns the out-state and, for
    a conditional vcc branch whose condition is a known constant, whether it is taken (True / False / None)."""
    pend, sc = dict(state[0]), dict(state[1])
    nops = 0
    taken = None
    for ln, raw, op, toks, in_asm in block["ins"]:
        if in_asm:
            if op.startswith("v_mfma"):
                for r in vregs(toks[0]):
                    pend[r] = ln
            elif op == "s_nop":
                nops += int(toks[0]) + 1
                if nops >= 18:
                    pend.clear()
            continue
        nops = 0
        if op.startswith(("v_", "ds_", "buffer_", "global_", "flat_", "scratch_")):
            used = set()
            for t in toks:
                used |= vregs(t)
            hit = sorted(r for r in used if r in pend)
            if hit and report is not None:
                report.append((ln, pend[hit[0]], raw))
        # scalar constant tracking (the structurised control flow's Flow blocks branch on s_mov'd masks)
        if op.startswith("s_") and toks:
            dst = "vcc" if toks[0] == "vcc" else sregs(toks[0])
            if op == "s_mov_b64" and dst is not None and toks[1] in ("0", "-1"):
                sc[dst] = int(toks[1])
            elif op in ("s_andn2_b64", "s_and_b64") and toks[0] == "vcc" and toks[1] == "exec":
                src = sregs(toks[2])
                v = sc.get(src)
                if v is None:
                    sc.pop("vcc", None)
                else:  # exec is non-zero in any block a wave executes
                    sc["vcc"] = (v == 0) if op == "s_andn2_b64" else (v != 0)
            elif dst is not None:
                sc.pop(dst, None)
            if op == "s_cbranch_vccnz" and "vcc" in sc:
                taken = bool(sc["vcc"])
            elif op == "s_cbranch_vccz" and "vcc" in sc:
                taken = not sc["vcc"]
        if op.startswith(("v_cmp", "v_cmpx")) or (op.startswith("s_") and toks and toks[0] == "vcc" and "andn2" not in op
                                                   and op not in ("s_and_b64",)):
            if op.startswith("v_cmp"):
                sc.pop("vcc", None)
    return (pend, sc), taken


def lint(lines):
    blocks = parse(lines)
    index = {b["label"]: k for k, b in enumerate(blocks) if b["label"]}

    def succs(k, taken):
        b = blocks[k]
        out = []
        tgt = [index[t] for t in b["succ"] if t in index]
        last = b["ins"][-1][2] if b["ins"] else ""
        if last in BRANCH_C and taken is not None:
            return tgt if taken else ([k + 1] if k + 1 < len(blocks) else [])
        out += tgt
        if b["fall"] and k + 1 < len(blocks):
            out.append(k + 1)
        return out

    # states are split by the known scalar constants (the structurised Flow blocks test masks set on each path), and
    # the pending sets of states with equal constants are merged
    state_in = [dict() for _ in blocks]  # block -> {frozen scalar constants: pending}
    state_in[0][frozenset()] = {}
    work = [(0, frozenset())]
    while work:
        k, key = work.pop(0)
        out, taken = transfer(blocks[k], (state_in[k][key], dict(key)), None)
        nkey = frozenset(out[1].items())
        for s_ in succs(k, taken):
            cur = state_in[s_].get(nkey)
            if cur is None:
                state_in[s_][nkey] = dict(out[0])
                work.append((s_, nkey))
                continue
            changed = False
            for r, ln in out[0].items():
                if r not in cur:
                    cur[r] = ln
                    changed = True
            if changed and (s_, nkey) not in work:
                work.append((s_, nkey))
    report = []
    for k, b in enumerate(blocks):
        for key, pend in state_in[k].items():
            transfer(b, (pend, dict(key)), report)
    return sorted(set(report))


def main():
    path = sys.argv[1]
    sym = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().split("\n")
    if sym:
        start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
        end = next((i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end")), len(lines))
        lines = lines[start:end + 1]
    probs = lint(lines)
    for ln, src, text in probs[:40]:
        print(f"line {ln}: touches an asm-MFMA result (written at line {src}) before its pad: {text}")
    print(f"{len(probs)} hazard(s)")
    return 1 if probs else 0


if __name__ == "__main__":
    sys.exit(main())
