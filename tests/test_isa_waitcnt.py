"""Build-time check of the hand-counted LDS-DMA waits (tests/isa_waitcnt_lint.py) over every shipped kernel that moves
operands by LDS-DMA: the compiled gfx950 ISA is walked path by path, and every `buffer_load ... lds` must be retired by
the hand-written `s_waitcnt vmcnt(N)` its lag names (`; dma-lag K` in the asm, default 1) before the barrier behind it.
Compiles for gfx950 on the CPU (no GPU needed).

The fixture tests/golden/isa/rdb_chain_rr0_f5c288c.s.gz is the round-5 RDB chain build the lint was written for: its
waits counted two row stores per step, and on steps that store no row of the strip hipcc deleted the first store as dead
(both at the same out-of-range offset), leaving the previous-but-one base row's DMA in flight when its readers read it
(DESIGN.md 3.7).  The lint must flag it; the shipped chain counts only its own DMA pieces and must be clean."""
import gzip
import os
from concurrent.futures import ProcessPoolExecutor

import pytest

from tests.isa_waitcnt_lint import annotate, kernels, lint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the translation units with LDS-DMA kernels (conv_wgrad.hip: the LDS-DMA weight gradients conv_wgrad64_glds*)
SOURCES = ["conv_dma.hip", "conv_wr.hip", "rdb_chain_narrow.hip", "conv_wgrad.hip"]
EXPECT = {"conv_dma.hip": ("conv_fwd_dma_kernel", "conv_fwd_s2_dma_kernel"), "conv_wr.hip": ("conv_wr_kernel",),
          "rdb_chain_narrow.hip": ("rdb_chain_rr_kernel",), "conv_wgrad.hip": ("conv_wgrad64_glds_kernel", "conv_wgrad64_glds_s2_kernel")}


def _lint_one(item):
    name, lines = item
    return name, lint(lines)


@pytest.mark.parametrize("src", SOURCES)
def test_shipped_lds_dma_waits_retire_their_pieces(gfx950_isa, src):
    ks = {n: ls for n, ls in kernels(gfx950_isa[src]).items() if annotate(ls)}
    for stem in EXPECT[src]:  # every LDS-DMA kernel of the file is found (a rename would silently skip it)
        assert any(stem in n for n in ks), (stem, list(ks))
    # the lint is pure Python: one process per kernel (the conv_fwd_dma<0> walks are the long ones)
    items = sorted(ks.items(), key=lambda kv: -len(kv[1]))
    with ProcessPoolExecutor(min(os.cpu_count() or 1, 8, len(ks))) as ex:
        res = dict(ex.map(_lint_one, items))
    bad = {n: r[:3] for n, r in res.items() if r}
    print(f"{src}: {len(ks)} LDS-DMA kernels, {sum(len(annotate(ls)) for ls in ks.values())} DMA instructions linted")
    assert not bad, bad


def test_lint_flags_the_round5_chain_form():
    """The f5c288c chain (base rows requested two steps ahead, lag 2): the dead-store-eliminated step leaves a base row's
    DMA in flight at the hand wait that must retire it."""
    with gzip.open(os.path.join(ROOT, "tests", "golden", "isa", "rdb_chain_rr0_f5c288c.s.gz"), "rt") as f:
        ks = kernels(f.read())
    assert len(ks) == 1
    (lines,) = ks.values()
    races = lint(lines, default_lag=2)
    assert races, "the lint must flag the round-5 chain's hand-counted wait"
    assert all(b >= 2 for _w, _d, b in races)


def test_lint_counts_paths_not_source():
    """Synthetic: a DMA, then a branch that issues two stores on one side and one on the other (what dead-store
    elimination did to the round-5 chain), then a hand wait vmcnt(2) that assumes two: flagged; with two on both sides,
    clean."""
    def isa(one_side):
        return f"""_Zkernel_test:
\t;;#ASMSTART
\tbuffer_load_dwordx4 v1, s[0:3], 0 offen lds
\t;;#ASMEND
\ts_cmp_eq_u32 s4, 0
\ts_cbranch_scc1 .LBB0_2
\tbuffer_store_dwordx2 v[2:3], v4, s[8:11], 0 offen
\tbuffer_store_dwordx2 v[2:3], v5, s[8:11], 0 offen
\ts_branch .LBB0_3
.LBB0_2:
\tbuffer_store_dwordx2 v[2:3], v4, s[8:11], 0 offen
{'' if one_side else chr(9) + 'buffer_store_dwordx2 v[2:3], v5, s[8:11], 0 offen'}
.LBB0_3:
\t;;#ASMSTART
\ts_waitcnt vmcnt(2)
\t;;#ASMEND
\ts_barrier
\ts_endpgm
.Lfunc_end0:
""".split("\n")
    races = lint(isa(True))
    assert len(races) == 1 and races[0][1] == 3, races  # (wait line, DMA line 3, hand wait 1)
    assert lint(isa(False)) == []
