"""Deterministic OSGPS register-level scenarios shared by the oracle, golden and
GPU parity tests.

A scenario is a list of correlator calls; before each call a few register
writes happen (the way osgpsisr.c's acquisition / pull-in / tracking states
drive ch_carrier, ch_code, ch_code_slew, ch_epoch_load and ch_cntl).  The IF
is synthesised with integer arithmetic only (numpy PCG64 + an 8-phase integer
LO), so every platform regenerates byte-identical input.

`run(osg, scn)` drives any object with the gp2021.c accessor names
(OracleOSG, RefOSG, gnsscorr.OSG) and returns REG_read after every call plus
the final correlator state when the object exposes it.
"""
from __future__ import annotations

import numpy as np

LO8 = np.array([[-1, 2], [1, 2], [2, 1], [2, -1], [1, -2], [-1, -2], [-2, -1], [-2, 1]],
               np.int64)


def _ca_chips(prn: int) -> np.ndarray:
    """ICD C/A chips (0/1) via the G2 delay table (GPS IS-200 Table 3-Ia)."""
    g2s = [5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470, 471,
           472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862]
    g1 = np.zeros(1023, np.int64)
    g2 = np.zeros(1023, np.int64)
    r1 = [1] * 10
    r2 = [1] * 10
    for i in range(1023):
        g1[i] = r1[9]
        g2[i] = r2[9]
        f1 = r1[2] ^ r1[9]
        f2 = r2[1] ^ r2[2] ^ r2[5] ^ r2[7] ^ r2[8] ^ r2[9]
        r1 = [f1] + r1[:9]
        r2 = [f2] + r2[:9]
    return g1 ^ np.roll(g2, g2s[prn - 1])


def synth_if(nsamp: int, seed: int, sigs=(), full_range: bool = False, iq: bool = True,
             fs_num: int = 16368, if_word: int = 635008600) -> np.ndarray:
    """Integer-only IF.  sigs: (prn, code_phase_samples, carrier_word_offset, amplitude)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n = np.arange(nsamp, dtype=np.int64)
    if full_range:
        raw = rng.integers(-128, 128, size=(nsamp, 2 if iq else 1), dtype=np.int64)
        return raw.astype(np.int8).reshape(-1)
    noise = rng.integers(-5, 6, size=(nsamp, 2), dtype=np.int64)
    acc = noise * 4
    for prn, cp, dw, amp in sigs:
        chips = _ca_chips(prn)
        # 16 samples per chip at 16.368 Msps
        c = 2 * chips[((n + cp) // 16) % 1023] - 1
        ph = (n * (if_word + dw)) & 0xFFFFFFFF
        lo = LO8[(ph >> 29).astype(np.int64)]
        acc[:, 0] += amp * c * lo[:, 0]
        acc[:, 1] += amp * c * lo[:, 1]
    # 2-bit quantiser {-3,-1,1,3} with threshold 8
    q = np.where(acc >= 0, np.where(acc < 8, 1, 3), np.where(acc > -8, -1, -3))
    if not iq:
        q = q[:, :1]
    return q.astype(np.int8).reshape(-1)


def make_scenario(name: str, seed: int, n_calls: int, nsamp: int = 8380, full_range=False,
                  iq=True, heavy_slew=False, prns=None, carrier_ref=31750430, code_ref=6710886,
                  tic_period=0.0):
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    nch = 12
    if prns is None:
        prns = [int(p) for p in rng.integers(1, 33, size=nch)]
        prns[0] = 32      # exercise the row over-read past the last PRN
        prns[3] = 0       # one idle channel
    sigs = [(p, int(rng.integers(0, 16368)), int(rng.integers(-2000, 2000)) * 20, 3)
            for p in prns[:6] if p > 0]
    IF = synth_if(nsamp * n_calls, seed, sigs, full_range=full_range, iq=iq)
    ops = []   # list per call of (method, args)
    first = []
    for ch in range(nch):
        first.append(("ch_carrier", ch, carrier_ref + int(rng.integers(-80000, 80000))))
        first.append(("ch_code", ch, code_ref + int(rng.integers(-40, 40))))
        first.append(("ch_cntl", ch, prns[ch]))
    for k in range(n_calls):
        cur = list(first) if k == 0 else []
        for ch in range(nch):
            u = rng.random()
            if u < 0.25:
                cur.append(("ch_carrier", ch, carrier_ref + int(rng.integers(-80000, 80000))))
            elif u < 0.45:
                cur.append(("ch_code", ch, code_ref + int(rng.integers(-200, 200))))
            elif u < 0.55:
                s = int(rng.integers(0, 2046)) if heavy_slew else int(rng.integers(0, 3))
                cur.append(("ch_code_slew", ch, s))
            elif u < 0.58:
                cur.append(("ch_epoch_load", ch, int(rng.integers(0, 0x10000))))
            elif u < 0.60 and ch != 0:
                cur.append(("ch_cntl", ch, int(rng.integers(0, 33))))
            elif u < 0.605 and heavy_slew:
                cur.append(("ch_code_slew", ch, int(rng.integers(2046, 65536))))
            elif u < 0.62 and heavy_slew:
                cur.append(("ch_code", ch, int(rng.integers(0, 1 << 26))))
        ops.append(cur)
    return dict(name=name, nsamp=nsamp, n_calls=n_calls, IF=IF, ops=ops, iq=iq,
                tic_period=tic_period)


SCENARIOS = {
    # 12 channels, planted signals, small slews: the tracking regime
    "track12": dict(seed=11, n_calls=40),
    # full-range int8 input, large slews (over-read into the next rows/tables),
    # arbitrary code words (several dumps per call)
    "wild": dict(seed=23, n_calls=24, full_range=True, heavy_slew=True),
    # I-only processing (use_iq_processing = 0)
    "ionly": dict(seed=37, n_calls=16, iq=False, full_range=True, heavy_slew=True),
    # 1-ms calls (16368 samples) as used by the batched API
    "ms1": dict(seed=41, n_calls=20, nsamp=16368),
    # TIC latch every 0.01 s at fs = 16.0 MHz (reference tic_ref = SAMP_RATE*tic_period)
    "tic": dict(seed=53, n_calls=48, nsamp=8192, tic_period=0.004),
}


def get(name: str):
    return make_scenario(name, **SCENARIOS[name])


def run(osg, scn, state_every=False):
    """Apply a scenario to an OSG-like object; returns (reg_read[n_calls,256], states)."""
    nsamp = scn["nsamp"]
    bps = 2 if scn["iq"] else 1
    IF = scn["IF"]
    regs = np.zeros((scn["n_calls"], 256), np.int32)
    states = []
    for k, cur in enumerate(scn["ops"]):
        for op in cur:
            getattr(osg, op[0])(*op[1:])
        chunk = IF[k * nsamp * bps:(k + 1) * nsamp * bps]
        osg.sim(chunk, nsamp)
        regs[k] = np.asarray(osg.REG_read[:256], np.int32)
        if state_every and hasattr(osg, "chan_state"):
            states.append(osg.chan_state())
    final = osg.chan_state() if hasattr(osg, "chan_state") else None
    return regs, (states if state_every else final)
