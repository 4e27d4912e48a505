"""The reference's recorded SoftGNSS tracking runs as test inputs.

tests/golden/sgt_trackres.npz holds trackResults(1), the numeric settings and
channel(1) of SCI/GLONASS/L1/trackingResults.dat and L2/trackingResults.dat
(made by tests/golden/make_sgt_trackres_golden.py through oracle/scilab_save.py).

Both runs used the tracking.sci variants that the current file keeps as
comments: codeFreq = codeFreqBasis - codeNco (tracking.sci:366, no carrier
aiding) and absoluteSample = mtell(fid)/dataAdaptCoeff (:379).  Their mseek
took skipNumberOfBytes as a sample count (absoluteSample(1) = skip +
codePhase - 1 + blksize(1): L1 16 000 000 + 14 912 + 16 000 = 16 030 912).

Tolerances, used by the CPU (oracle) and GPU (sgt.hip) replays alike:
  * blksize, absoluteSample, codeFreq, dllDiscr, dllDiscrFilt: bit-exact
    (sqrt, division and the DLL filter are correctly rounded IEEE fp64);
  * pllDiscr = atan(Q_P/I_P)/(2 pi): within 1e-15 relative (the libm atan of
    the Scilab build and ours differ in the last ulp in about a third of the
    epochs);
  * pllDiscrFilt, the running carrier NCO that such ulps feed: within 1e-12
    of the run's largest |pllDiscrFilt| (its terms are k1*carrError ~ 10-60 Hz,
    so its error is absolute, not relative to a value that crosses zero);
  * carrFreq = carrFreqBasis + carrNco: within 1e-15 relative.
"""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sgt_trackres.npz")
RUNS = ("L1", "L2")
SUMS = ("I_E", "I_P", "I_L", "Q_E", "Q_P", "Q_L")
EXACT = ("absoluteSample", "codeFreq", "dllDiscr", "dllDiscrFilt")


def load():
    return np.load(GOLDEN)


def run_inputs(z, run):
    """(settings dict of the record, FCH, acquiredFreq, codePhase, skip, sums [n, 6])."""
    st = dict(zip(list(z["settings_names"]), z[f"{run}_settings"].tolist()))
    fch, acq_freq, code_phase = z[f"{run}_chan"].tolist()
    sums = np.stack([z[f"{run}_{k}"] for k in SUMS], 1)
    return st, int(fch), acq_freq, int(code_phase), int(st["skipNumberOfBytes"]), sums


def scilab_settings(st):
    """The record's settings under the sgt_oracle / gnsscorr.sgt_cfg names, with
    the variants the record shows."""
    return dict(samplingFreq=st["samplingFreq"], codeFreqBasis=st["codeFreqBasis"],
                codeLength=int(st["codeLength"]), IF=st["IF"], L1_IF_step=st["L1_IF_step"],
                fileType=int(st["fileType"]), dllCorrelatorSpacing=st["dllCorrelatorSpacing"],
                dllNoiseBandwidth=st["dllNoiseBandwidth"], dllDampingRatio=st["dllDampingRatio"],
                pllNoiseBandwidth=st["pllNoiseBandwidth"],
                fllNoiseBandwidth=st["fllNoiseBandwidth"], codeNcoVariant=1, absSampleVariant=1)


def check_against_record(z, run, got, blksize):
    """Assert a replay (dict of per-epoch arrays) against the recorded run."""
    st, fch, _, code_phase, skip, _ = run_inputs(z, run)
    rec_abs = z[f"{run}_absoluteSample"]
    want_blk = np.diff(np.r_[skip + code_phase - 1, rec_abs]).astype(np.int64)
    np.testing.assert_array_equal(np.asarray(blksize, np.int64), want_blk)
    for k in EXACT:
        np.testing.assert_array_equal(got[k], z[f"{run}_{k}"], err_msg=f"{run} {k}")
    pd, pdw = np.asarray(got["pllDiscr"]), z[f"{run}_pllDiscr"]
    assert np.all(np.abs(pd - pdw) <= 1e-15 * np.abs(pdw)), f"{run} pllDiscr"
    pf, pfw = np.asarray(got["pllDiscrFilt"]), z[f"{run}_pllDiscrFilt"]
    assert np.max(np.abs(pf - pfw)) <= 1e-12 * np.max(np.abs(pfw)), f"{run} pllDiscrFilt"
    cf, cfw = np.asarray(got["carrFreq"]), z[f"{run}_carrFreq"]
    assert np.all(np.abs(cf - cfw) <= 1e-15 * np.abs(cfw)), f"{run} carrFreq"
