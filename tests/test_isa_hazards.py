"""Build-time check of the kernels that issue MFMAs from inline asm (csrc/mfma_agpr.h): hipcc inserts no wait states
around them, so the compiled gfx950 ISA is linted (tests/isa_mfma_lint.py) for any instruction that touches an asm
MFMA's destination registers before the kernel's hazard pad, on every control-flow path.  Compiles for gfx950 on the
CPU (no GPU needed)."""
import re

import pytest

from tests.isa_mfma_lint import lint


def _kernels(asm_text):
    lines = asm_text.split("\n")
    out = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w*kernel\w*):", l)
        if m:
            end = next((j for j in range(i + 1, len(lines)) if lines[j].startswith(".Lfunc_end")), len(lines))
            out[m.group(1)] = lines[i:end + 1]
    return out


@pytest.mark.parametrize("src", ["rdb_chain.hip", "conv_wr.hip", "srcnn.hip"])
def test_asm_mfma_results_are_padded(src, gfx950_isa):
    kern = _kernels(gfx950_isa[src])
    assert kern, "no kernels found in the ISA"
    bad = {name: lint(lines)[:5] for name, lines in kern.items()}
    bad = {k: v for k, v in bad.items() if v}
    assert not bad, bad
