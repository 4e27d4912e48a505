"""Source-level regression pins (CPU).

Round 2's wrong tracking sums came from an inline-asm v_mad_i32_i24: an
INLINEASM statement carries no implicit EXEC operand, so machine passes may
move a non-volatile asm across the exec-mask writes of divergent branches,
where it writes lanes a branch had masked off (profiles/r3/mad24_hazard_repro_r3.log,
DESIGN.md section 3).  Every inline asm in the device sources must be volatile.
The repro form (TRACK_ASM_MAD) and the other measured-out tracking switches
(TRACK_SLOTS > 1 with its inline-asm slot read, TRACK_DMA_AUX, GNSSCORR_TRACK_V1,
TRACK_LOAD4) were removed in round 6; git history keeps them.
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
        for i, line in enumerate(lines, 1):
            t = line.strip()
            if re.search(r"\basm\s*\(", t):
                bad.append(f"{f}:{i}: {t}")
    assert not bad, "non-volatile inline asm:\n" + "\n".join(bad)


def test_measured_out_switches_are_gone():
    gone = ("TRACK_ASM_MAD", "TRACK_SLOTS", "TRACK_DMA_AUX", "GNSSCORR_TRACK_V1", "TRACK_LOAD4")
    for f, lines in _sources():
        text = "\n".join(lines)
        for g in gone:
            assert g not in text, (f, g)
