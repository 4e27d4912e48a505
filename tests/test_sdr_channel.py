"""CPU: the GPS-SDR Channel fixtures and host code.

The oracle for this row is the reference Channel class itself, compiled from
objects/channel.cpp (oracle/_ref/libsdr_chan_ref.so, oracle/sdr_chan_ref.cpp);
tests/golden/sdr_channel.npz holds its outputs on the synthetic navigation
streams of tests/sdr_nav_scenarios.py (make_sdr_chan_golden.py).
Checked here: the ICD-200 parity encoder against the reference ParityCheck,
the product's host Channel::Start against the reference object byte for byte,
the scenario inputs against their pinned SHA-256, and the fixture against the
reference build.
"""
import hashlib
import os

import numpy as np
import pytest

import sdr_nav_scenarios as N
import sdr_oracle as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
need_ref = pytest.mark.skipif(not S.have_ref_chan(), reason="reference build (oracle/_ref) absent")


def _golden():
    return np.load(os.path.join(GOLD, "sdr_channel.npz"))


def test_parity_encoder_roundtrip():
    rng = np.random.default_rng(4)
    prev = 0
    for _ in range(500):
        w = N.encode_word(int(rng.integers(0, 1 << 24)), prev)
        u = w | (prev & 3) << 30                 # bits 31-30: D29*, D30* (BitStuff layout)
        if u & 0x40000000:
            u ^= 0x3FFFFFC0
        assert N.parity_ok(u)
        assert not N.parity_ok(u ^ (1 << int(rng.integers(6, 30))))   # any single data-bit error
        prev = w


@need_ref
def test_parity_against_reference():
    ref = S.RefSdrChannel(0)
    rng = np.random.default_rng(5)
    for _ in range(300):
        w = int(rng.integers(0, 1 << 32, dtype=np.uint64))
        assert ref.parity(w) == N.parity_ok(w)


def test_scenario_inputs_pinned():
    import make_sdr_chan_golden as G
    g = _golden()
    for k, sc in enumerate(N.SCENARIOS):
        corr = G.scenario_corr(sc, int(g["n_ms"]))
        assert hashlib.sha256(corr.tobytes()).hexdigest() == str(g["corr_sha256"][k])


@need_ref
def test_host_start_matches_reference(gc):
    ref = S.RefSdrChannel(3)
    for sv, dop, cl, *_ in N.SCENARIOS + [(31, -14999, 20, 0, 0, 0, 0, 0)]:
        ref.start(sv, dop, cl)
        mine = gc.SdrCorrCtx.channel_start(3, sv, dop, cl)
        assert mine.tobytes()[:580] == ref.state().tobytes()[:580]


@need_ref
def test_golden_matches_reference_build():
    import make_sdr_chan_golden as G
    g = _golden()
    k = 0
    sc = N.SCENARIOS[k]
    corr = G.scenario_corr(sc, int(g["n_ms"]))
    ref = S.RefSdrChannel(k)
    ref.start(int(sc[0]), int(sc[1]), int(sc[2]))
    fb, subs, st = ref.run(corr)
    assert (G.flags_of(fb) == g["flags"][k]).all()
    assert st.tobytes() == g["state"][k].tobytes()
    rows = g["sub_rows"][g["sub_rows"][:, 0] == k]
    assert [m for m, _ in subs] == list(rows[:, 1])
