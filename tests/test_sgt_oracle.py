"""CPU: the SoftGNSS float-tracking oracle (oracle/sgt_oracle.py) and the
host-side pieces of the sgt C-ABI that need no GPU.

Reference: POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/tracking.sci:150-400,
GPS/L1/tracking.sci:124-360, calcLoopCoef.sci:39-43, calcFLLPLLLoopCoef.sci:36-38.
Parity unpinned against a Scilab run (no interpreter in the image):
the oracle is pinned by planted-signal tracking KATs (lock, frequency, code
alignment) below.
"""
import math

import numpy as np
import pytest

import sgt_oracle as S

FS = 16e6


def _glo_start(cp_chips, fs=FS):
    """1-based code phase of the first ST-code start for a signal whose chip
    phase at sample 0 is cp_chips (what acquisition.sci would report)."""
    return int(round((511 - cp_chips) / 0.511e6 * fs)) + 1


def test_loop_coefficients_match_scilab_formulae(gc):
    for system in (0, 1):
        cfg = gc.sgt_cfg(system)
        tau1, tau2, k1, k2, k3 = _coefs(gc, cfg)
        s = S.settings(system)
        rt1, rt2 = S.calc_loop_coef(s["dllNoiseBandwidth"], s["dllDampingRatio"], 1.0)
        rk = S.calc_fll_pll_loop_coef(s["pllNoiseBandwidth"], s["fllNoiseBandwidth"], 0.001)
        assert (tau1, tau2) == (rt1, rt2)
        assert (k1, k2, k3) == rk
    # the hand values of calcFLLPLLLoopCoef for 25 Hz / 250 Hz / 1 ms
    k1, k2, k3 = S.calc_fll_pll_loop_coef(25.0, 250.0, 0.001)
    assert math.isclose(k2, 1.414 * 25 / 0.53) and math.isclose(k3, 1.0)


def _coefs(gc, cfg):
    import ctypes as C
    v = [C.c_double() for _ in range(5)]
    gc.lib().gnsscorr_sgt_loop_coefs(C.byref(cfg), *[C.byref(x) for x in v])
    return tuple(x.value for x in v)


def test_init_chan_follows_tracking_sci(gc):
    cfg = gc.sgt_cfg(1)
    out = np.zeros(1, gc.SGT_CHAN)
    assert gc.lib().gnsscorr_sgt_init_chan(cfg, 3, 2, 1000, 777, 2.6e6, out.ctypes.data) == 0
    c = out[0]
    assert c["pos"] == 1000 + 777 - 1 and c["stream"] == 2 and c["code_id"] == 3
    assert c["code_freq"] == 0.511e6 and c["carr_freq"] == c["carr_freq_basis"] == 2.6e6
    assert c["i1"] == c["q1"] == 0.001 and c["rem_code"] == 0 and c["status"] == 0
    # bad FCH / PRN / code phase are rejected
    assert gc.lib().gnsscorr_sgt_init_chan(cfg, 7, 0, 0, 1, 0.0, out.ctypes.data) != 0
    assert gc.lib().gnsscorr_sgt_init_chan(gc.sgt_cfg(0), 33, 0, 0, 1, 0.0,
                                           out.ctypes.data) != 0
    assert gc.lib().gnsscorr_sgt_init_chan(cfg, 0, 0, 0, 0, 0.0, out.ctypes.data) != 0
    bad = gc.sgt_cfg(1, codeLength=1023)
    assert gc.lib().gnsscorr_sgt_init_chan(bad, 0, 0, 0, 1, 0.0, out.ctypes.data) != 0


def test_padded_code_layout():
    c = S.padded_code(1)
    st = S.generate_st_code()
    assert len(c) == 513 and c[0] == st[-1] and c[-1] == st[0] and (c[1:-1] == st).all()
    g = S.padded_code(0, 5)
    assert len(g) == 1025


def test_correlate_epoch_bookkeeping(gc):
    s = S.settings(1)
    IF = gc.ifgen(40000, [], fs=FS, seed=1)
    pad = S.padded_code(1)
    r = S.correlate(IF, s, pad, 5, 0.3, 1.0, 0.511e6 + 3.0, 1.2e6)
    sums, blk, pos, rc, rcar = r
    step = (0.511e6 + 3.0) / FS
    assert blk == math.ceil((511 - 0.3) / step) and pos == 5 + blk
    assert 0 <= rc < step and -2 * math.pi < rcar < 2 * math.pi
    # out of data -> None (tracking.sci:273-277)
    assert S.correlate(IF, s, pad, 40000 - 100, 0.0, 0.0, 0.511e6, 1e6) is None


@pytest.mark.parametrize("fch,dop", [(-7, -2000.0), (0, 500.0), (6, 3100.0)])
def test_glonass_planted_signal_locks(gc, fch, dop):
    s = S.settings(1, samplingFreq=FS)
    cp = 123.4
    IF = gc.ifgen(int(FS * 0.2), [dict(system=1, fch=fch, code_phase=cp, doppler=dop, cn0=50.0,
                                       data_bits=0)], fs=FS, if_glo=1e6, seed=9)
    base = 1e6 + 0.5625e6 * fch
    r = S.track(IF, s, fch, _glo_start(cp), base + dop + 5.0, 180)
    assert len(r["I_P"]) == 180
    tail = slice(120, None)
    # Costas lock: the prompt energy sits on one arm; carrier within a few Hz
    assert np.median(np.abs(r["I_P"][tail])) > 5 * np.median(np.abs(r["Q_P"][tail]))
    assert abs(np.mean(r["carrFreq"][tail]) - (base + dop)) < 5.0
    assert (r["blksize"] >= 15990).all() and (r["blksize"] <= 16010).all()
    # prompt beats early and late on average (code aligned)
    p = np.hypot(r["I_P"][tail], r["Q_P"][tail]).mean()
    assert p > np.hypot(r["I_E"][tail], r["Q_E"][tail]).mean()
    assert p > np.hypot(r["I_L"][tail], r["Q_L"][tail]).mean()


def test_gps_planted_signal_locks(gc):
    s = S.settings(0, samplingFreq=FS)
    cp = 300.25
    IF = gc.ifgen(int(FS * 0.15), [dict(system=0, prn=11, code_phase=cp, doppler=-1500.0,
                                        cn0=50.0, data_bits=0)], fs=FS, if_gps=2.42e6, seed=4)
    start = int(round((1023 - cp) / 1.023e6 * FS)) + 1
    r = S.track(IF, s, 11, start, 2.42e6 - 1500.0 - 8.0, 140)
    tail = slice(90, None)
    assert np.median(np.abs(r["I_P"][tail])) > 5 * np.median(np.abs(r["Q_P"][tail]))
    assert abs(np.mean(r["carrFreq"][tail]) - (2.42e6 - 1500.0)) < 5.0
