"""CPU: pin the scalar C restatement (oracle/osg_corr.c) of Sim_GP2021_int.

* against the committed golden fixtures produced by the reference itself
  (tests/golden/make_osg_golden.py, reference correlator.c:148-316), and
* against oracle/_ref/libosg_ref.so directly when the reference is present.
"""
import ctypes as C
import hashlib
import os

import numpy as np
import pytest

import osg_scenarios as S

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("name", list(S.SCENARIOS))
def test_oracle_matches_golden(oracle, name):
    scn = S.get(name)
    g = np.load(os.path.join(GOLD, f"osg_{name}.npz"))
    assert hashlib.sha256(scn["IF"].tobytes()).hexdigest() == str(g["if_sha256"])
    o = oracle.OracleOSG(12, scn["iq"], 16.0e6, scn["tic_period"])
    regs, st = S.run(o, scn)
    np.testing.assert_array_equal(regs, g["reg_read"])
    for k in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
        np.testing.assert_array_equal(st[k], g[k], err_msg=k)


def test_golden_exercises_quirks():
    """The fixtures must actually cover the hard parts (SURVEY 7 'Hard parts')."""
    g = np.load(os.path.join(GOLD, "osg_wild.npz"))
    assert (g["reg_read"][:, 0x82] != 0).sum() > 10            # dumps happen
    t = np.load(os.path.join(GOLD, "osg_tic.npz"))
    assert (t["reg_read"][:, 0x83] == 0x2000).sum() > 3        # TIC latches
    # accumulators wrap to int16 in from_gps (gp2021.c:24-28): values beyond short exist
    big = np.abs(g["reg_read"][:, 0x84:0xE4]).max()
    assert big > 32767


@pytest.mark.skipif(not os.path.isdir("/root/reference"), reason="reference not mounted")
@pytest.mark.parametrize("name", ["track12", "wild"])
def test_oracle_matches_reference_build(oracle, name):
    oracle.build(ref=True)
    scn = S.get(name)
    o = oracle.OracleOSG(12, scn["iq"], 16.0e6, scn["tic_period"])
    r1, s1 = S.run(o, scn)
    ref = oracle.RefOSG(12, scn["tic_period"])
    C.c_int.in_dll(ref.L, "use_iq_processing").value = 1 if scn["iq"] else 0
    ref.L.correlator_init(scn["tic_period"])
    r2, s2 = S.run(ref, scn)
    np.testing.assert_array_equal(r1, r2)
    for k in s2:
        np.testing.assert_array_equal(s1[k], s2[k], err_msg=k)


def test_oracle_words_16368():
    import osg_oracle
    w = osg_oracle.osg_words(16.368e6)
    assert (w["carrier_ref"], w["code_ref"], w["d_freq"]) == (31750430, 6710886, 13120)
    w = osg_oracle.osg_words(16.0e6)
    assert (w["carrier_ref"], w["code_ref"], w["d_freq"]) == (32480690, 6865236, 13421)
