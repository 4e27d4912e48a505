"""oracle/sgt_oracle.py -- TEST INFRASTRUCTURE ONLY.

fp64 numpy restatement of the SoftGNSS ("sgt") float tracking loop of the
Scilab receivers, one channel at a time, line by line:

  GLONASS POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/tracking.sci:150-400
  GPS     POSTPROCESSING_SCILAB_RECEIVERS/GPS/L1/tracking.sci:124-360
  loop coefficients  GLONASS/L1/include/calcLoopCoef.sci:39-43,
                     GLONASS/L1/include/calcFLLPLLLoopCoef.sci:36-38

Per 1-code-period epoch: blksize = ceil((L - remCode)/step); E/P/L replicas
code[ceil(remCode -/+ spc + k*step) + 1] from the padded code [c(end) c c(1)];
carrier exp(i*((2*pi*f)*t + remCarr)); I = sum(code*imag(carr*raw)),
Q = sum(code*real(carr*raw)); then the FLL-assisted PLL and the DLL.

Assumptions: Scilab's `a:step:b` yields a + k*step (ImplicitList element
formula), and complex products/sums are plain IEEE fp64.

Parity status: the LOOP half (blksize / remCodePhase chain, FLL/PLL and DLL
discriminators and filters, carrFreq, codeFreq, absoluteSample) is PINNED to
the reference's own recorded runs: SCI/GLONASS/L1/trackingResults.dat and
L2/trackingResults.dat (1500 epochs each, written by postProcessing.sce:143),
replayed from their recorded sums by `replay` (tests/test_sgt_trackres.py):
codeFreq, dllDiscr, dllDiscrFilt and absoluteSample equal the record
bit-for-bit, carrFreq/pllDiscr/pllDiscrFilt to within the last-ulp atan
difference of the Scilab build.  Those runs used the tracking.sci variants now
commented out: codeFreq without carrier aiding (:366, `codeNcoVariant=1`)
and absoluteSample = mtell/dataAdaptCoeff (:379, `absSampleVariant=1`).  The
CORRELATOR half (the six sums) has no recorded input IF in the reference, so
it stays pinned by planted-signal KATs only (tests/test_sgt_oracle.py).
Only tests/, smoke() and bench.py's cpu_baseline use this module.
"""
from __future__ import annotations

import math

import numpy as np

from acq_oracle import generate_ca_code, generate_st_code

# trackResults fields per epoch, in the order the C-ABI record stores them
FIELDS = ("I_E", "I_P", "I_L", "Q_E", "Q_P", "Q_L", "carrFreq", "codeFreq", "absoluteSample",
          "dllDiscr", "dllDiscrFilt", "pllDiscr", "pllDiscrFilt")


def calc_loop_coef(lbw: float, zeta: float, k: float):
    """calcLoopCoef.sci:39-43 -> (tau1, tau2)."""
    wn = lbw * 8 * zeta / (4 * zeta ** 2 + 1)
    return k / (wn * wn), 2.0 * zeta / wn


def calc_fll_pll_loop_coef(pllbw: float, fllbw: float, T: float):
    """calcFLLPLLLoopCoef.sci:36-38 -> (k1, k2, k3)."""
    k1 = T * ((pllbw / 0.53) ** 2) + 1.414 * (pllbw / 0.53)
    k2 = 1.414 * (pllbw / 0.53)
    k3 = T * (fllbw / 0.25)
    return k1, k2, k3


def settings(system: int, **kw) -> dict:
    """initSettings.sci defaults (GLONASS/L1:41-107, GPS/L1:41-95), overridable."""
    if system == 1:
        s = dict(system=1, samplingFreq=16e6, codeFreqBasis=0.511e6, codeLength=511, IF=1e6,
                 L1_IF_step=0.5625e6, GLONASS_zero_channel=1602e6, dllCorrelatorSpacing=0.05,
                 dllNoiseBandwidth=0.5, dllDampingRatio=0.7, pllNoiseBandwidth=25.0,
                 fllNoiseBandwidth=250.0, fileType=2, switchIQ=0)
    else:
        s = dict(system=0, samplingFreq=16e6, codeFreqBasis=1.023e6, codeLength=1023, IF=2.42e6,
                 L1_IF_step=0.0, GLONASS_zero_channel=0.0, dllCorrelatorSpacing=0.2,
                 dllNoiseBandwidth=0.1, dllDampingRatio=0.7, pllNoiseBandwidth=25.0,
                 fllNoiseBandwidth=250.0, fileType=2, switchIQ=0)
    # tracking.sci variants (both 0 = the current file): codeNcoVariant 1 =
    # codeFreq = basis - codeNco (:366, no carrier aiding); absSampleVariant 1 =
    # absoluteSample = mtell(fid)/dataAdaptCoeff, the whole-sample position (:379)
    s.update(codeNcoVariant=0, absSampleVariant=0)
    s.update(kw)
    return s


def padded_code(system: int, prn: int = 1) -> np.ndarray:
    """tracking.sci:171-174 (GLONASS) / :140-142 (GPS): [c(end) c c(1)]."""
    c = generate_st_code() if system == 1 else generate_ca_code(prn)
    return np.concatenate([c[-1:], c, c[:1]])


def _raw(IF: np.ndarray, pos: int, n: int, s: dict) -> np.ndarray:
    if s["fileType"] == 1:
        return IF[pos:pos + n].astype(np.float64)
    v = IF[2 * pos:2 * (pos + n)].astype(np.float64)
    r1, r2 = v[0::2], v[1::2]
    if s["system"] == 1 and s["switchIQ"]:
        return r2 + 1j * r1
    return r1 + 1j * r2


def correlate(IF, s, code_pad, pos, rem_code, rem_carr, code_freq, carr_freq):
    """One epoch of the correlator block (GLONASS tracking.sci:245-327).
    Returns (sums[6] as I_E,I_P,I_L,Q_E,Q_P,Q_L, blksize, pos', remCode', remCarr')
    or None when the record has fewer than blksize samples left (:273-277)."""
    fs, L, spc = s["samplingFreq"], s["codeLength"], s["dllCorrelatorSpacing"]
    step = code_freq / fs
    blksize = int(math.ceil((L - rem_code) / step))
    n_avail = (len(IF) if s["fileType"] == 1 else len(IF) // 2) - pos
    if n_avail < blksize:
        return None
    raw = _raw(IF, pos, blksize, s)
    k = np.arange(blksize, dtype=np.float64)
    ks = k * step
    early = code_pad[np.ceil((rem_code - spc) + ks).astype(np.int64)]
    late = code_pad[np.ceil((rem_code + spc) + ks).astype(np.int64)]
    tP = rem_code + ks
    prompt = code_pad[np.ceil(tP).astype(np.int64)]
    rem_code_n = (tP[-1] + step) - L
    time = np.arange(blksize + 1, dtype=np.float64) / fs
    trig = ((carr_freq * 2.0 * np.pi) * time) + rem_carr
    last = trig[blksize]
    rem_carr_n = last - math.trunc(last / (2 * np.pi)) * (2 * np.pi)
    carr = np.exp(1j * trig[:blksize])
    bb = carr * raw
    qb, ib = bb.real, bb.imag
    sums = np.array([np.sum(early * ib), np.sum(prompt * ib), np.sum(late * ib),
                     np.sum(early * qb), np.sum(prompt * qb), np.sum(late * qb)])
    return sums, blksize, pos + blksize, rem_code_n, rem_carr_n


class Loop:
    """Per-channel loop state and the update after one epoch's sums
    (tracking.sci:179-201 initial values, :329-398 per epoch)."""

    def __init__(self, s, code_id, pos, acquired_freq):
        self.s = s
        self.tau1, self.tau2 = calc_loop_coef(s["dllNoiseBandwidth"], s["dllDampingRatio"], 1.0)
        self.k1, self.k2, self.k3 = calc_fll_pll_loop_coef(s["pllNoiseBandwidth"],
                                                           s["fllNoiseBandwidth"], 0.001)
        self.code_id = code_id
        self.pos = pos
        self.code_freq = s["codeFreqBasis"]
        self.rem_code = 0.0
        self.carr_freq = self.carr_basis = acquired_freq
        self.rem_carr = 0.0
        self.old_code_nco = self.old_code_err = self.old_carr_nco = self.old_carr_err = 0.0
        self.I1 = self.Q1 = 0.001

    def blksize(self):
        """tracking.sci:250-252."""
        step = self.code_freq / self.s["samplingFreq"]
        return int(math.ceil((self.s["codeLength"] - self.rem_code) / step)), step

    def advance(self, blk, step, rem_carr_n=None):
        """Carry-over of an epoch of blk samples (:258, :295-302, :309-310)."""
        tP_last = self.rem_code + float(blk - 1) * step
        self.rem_code = (tP_last + step) - self.s["codeLength"]
        self.pos += blk
        if rem_carr_n is not None:
            self.rem_carr = rem_carr_n

    def update(self, sums):
        """FLL-assisted PLL + DLL on one epoch's sums (:329-398); returns the record
        values in FIELDS order."""
        s = self.s
        I_E, I_P, I_L, Q_E, Q_P, Q_L = (float(x) for x in sums)
        I2, Q2 = self.I1, self.Q1
        self.I1, self.Q1 = I_P, Q_P
        cross = self.I1 * Q2 - I2 * self.Q1
        dot = abs(self.I1 * I2 + self.Q1 * Q2)
        freq_err = math.atan2(cross, dot) / math.pi
        carr_err = math.atan(Q_P / I_P) / (2.0 * math.pi)
        carr_nco = self.old_carr_nco + self.k1 * carr_err - self.k2 * self.old_carr_err - \
            self.k3 * freq_err
        self.old_carr_nco, self.old_carr_err = carr_nco, carr_err
        self.carr_freq = self.carr_basis + carr_nco
        aE = math.sqrt(I_E * I_E + Q_E * Q_E)
        aL = math.sqrt(I_L * I_L + Q_L * Q_L)
        code_err = (aE - aL) / (aE + aL)
        code_nco = self.old_code_nco + (self.tau2 / self.tau1) * (code_err - self.old_code_err) + \
            code_err * (0.001 / self.tau1)
        self.old_code_nco, self.old_code_err = code_nco, code_err
        if s["codeNcoVariant"] == 1:
            self.code_freq = s["codeFreqBasis"] - code_nco                      # :366
        elif s["system"] == 1:
            fch = self.code_id
            self.code_freq = s["codeFreqBasis"] - code_nco + \
                (self.carr_freq - (s["IF"] + s["L1_IF_step"] * fch)) / \
                ((s["GLONASS_zero_channel"] + fch * s["L1_IF_step"]) / s["codeFreqBasis"])
        else:
            self.code_freq = s["codeFreqBasis"] - code_nco + ((self.carr_freq - s["IF"]) / 1540)
        if s["absSampleVariant"] == 1:
            abs_sample = float(self.pos)                                         # :379
        else:
            abs_sample = self.pos - self.rem_code * (s["samplingFreq"] / 1000) / s["codeLength"]
        return (I_E, I_P, I_L, Q_E, Q_P, Q_L, self.carr_freq, self.code_freq, abs_sample,
                code_err, code_nco, carr_err, carr_nco)


def replay(sums, s, code_id, code_phase_1b, acquired_freq, skip=0):
    """The loop half of tracking.sci driven by given per-epoch sums [n, 6]
    (I_E, I_P, I_L, Q_E, Q_P, Q_L) instead of correlations of a record: blksize
    and remCodePhase chain, discriminators, filters, NCO frequencies and
    absoluteSample.  Pins the loop against a recorded trackResults."""
    lp = Loop(s, code_id, skip + code_phase_1b - 1, acquired_freq)
    out = {f: [] for f in FIELDS}
    out["blksize"] = []
    for row in np.asarray(sums, dtype=np.float64):
        blk, step = lp.blksize()
        lp.advance(blk, step)
        for f, v in zip(FIELDS, lp.update(row)):
            out[f].append(v)
        out["blksize"].append(blk)
    return {f: np.asarray(v) for f, v in out.items()}


def track(IF, s, code_id, code_phase_1b, acquired_freq, n_ms, skip=0):
    """tracking.sci per-channel loop for n_ms epochs.  code_id: GPS PRN or GLONASS FCH.
    Returns a dict of FIELDS arrays (length = epochs actually processed) + 'blksize'."""
    code_pad = padded_code(s["system"], code_id)
    lp = Loop(s, code_id, skip + code_phase_1b - 1, acquired_freq)   # mseek, :163-168
    out = {f: [] for f in FIELDS}
    out["blksize"] = []
    for _ in range(n_ms):
        r = correlate(IF, s, code_pad, lp.pos, lp.rem_code, lp.rem_carr, lp.code_freq,
                      lp.carr_freq)
        if r is None:
            break
        sums, blk, pos, rem_code, rem_carr = r
        lp.pos, lp.rem_code, lp.rem_carr = pos, rem_code, rem_carr
        for f, v in zip(FIELDS, lp.update(sums)):
            out[f].append(v)
        out["blksize"].append(blk)
    return {f: np.asarray(v) for f, v in out.items()}
