"""CPU: the reference receiver at 16.368 Msps (oracle/_ref/e2e_ref_16368, the
reference's correlator.c / gp2021.c / osgpsisr.c compiled from /root/reference)
reproduces the committed golden of BASELINE config 1 -- PRN 1 acquired,
pulled in and tracked for more than 10 s (tests/golden/e2e16368.json).
Skipped where the reference build is absent."""
import hashlib
import json
import os
import subprocess

import pytest

import e2e_scenarios as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF16 = os.path.join(ROOT, "oracle", "_ref", "e2e_ref_16368")


@pytest.mark.skipif(not os.path.exists(REF16), reason="reference build not present")
def test_reference_config1_golden(gc, tmp_path):
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "e2e16368.json")))["config1"]
    s = E.SCENARIOS["config1"]
    IF = E.make_if(gc, "config1")
    assert hashlib.sha256(IF.tobytes()).hexdigest() == gold["if_sha256"]
    IF.tofile(tmp_path / "if.bin")
    subprocess.run([REF16, str(tmp_path / "if.bin"), str(tmp_path / "t"), str(s["calls"]), "1"],
                   check=True, timeout=600)
    tr = (tmp_path / "t").read_bytes()
    assert hashlib.sha256(tr).hexdigest() == gold["trace_sha256"]
    (first, held), = E.summary(tr, 1)
    assert first > 0 and held > 10.0
