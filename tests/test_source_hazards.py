"""Source-level regression pins (CPU).

Round 2's wrong tracking sums came from an inline-asm v_mad_i32_i24: an
INLINEASM statement carries no implicit EXEC operand, so machine passes may
move a non-volatile asm across the exec-mask writes of divergent branches,
where it writes lanes a branch had masked off (profiles/r3/mad24_hazard_repro_r3.log,
DESIGN.md section 3).  Every inline asm in the device sources must be volatile;
the only exception is the repro form kept behind TRACK_ASM_MAD (off by default).
"""
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                    "gnss-sdr.ru_amd", "csrc")


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".h")):
            yield f, open(os.path.join(CSRC, f)).read().split("\n")


def test_inline_asm_is_volatile():
    bad = []
    for f, lines in _sources():
        guard = []   # stack of (macro, active-branch-is-repro)
        for i, line in enumerate(lines, 1):
            t = line.strip()
            m = re.match(r"#\s*if(n?def)?\s+(\w+)", t)
            if m:
                guard.append(m.group(2) == "TRACK_ASM_MAD" and m.group(1) == "def")
                continue
            if re.match(r"#\s*else", t) and guard:
                guard[-1] = False
                continue
            if re.match(r"#\s*endif", t) and guard:
                guard.pop()
                continue
            if re.search(r"\basm\s*\(", t) and not any(guard):
                bad.append(f"{f}:{i}: {t}")
    assert not bad, "non-volatile inline asm outside the TRACK_ASM_MAD repro:\n" + "\n".join(bad)


def test_repro_macro_is_off_by_default():
    mk = open(os.path.join(os.path.dirname(CSRC), "Makefile")).read()
    assert "TRACK_ASM_MAD" not in mk
