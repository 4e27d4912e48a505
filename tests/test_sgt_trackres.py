"""The SoftGNSS loop restatement (oracle/sgt_oracle.py) against the reference's
own recorded tracking runs, SCI/GLONASS/L1/trackingResults.dat and
L2/trackingResults.dat (postProcessing.sce:143; 1500 epochs of one GLONASS
channel each).  The recorded six sums drive the loop; every other recorded
field is the check (tolerances: tests/trackres_fixture.py).

Reference: GLONASS/L1/tracking.sci:248-302 (blksize / remCodePhase chain),
:329-351 (FLL-assisted PLL), :353-375 (DLL), :379 (absoluteSample, mtell form),
:366 (codeFreq without carrier aiding).
"""
import os

import numpy as np
import pytest

import scilab_save
import sgt_oracle as S
import trackres_fixture as TR

SCI = "/root/reference/trunk/GNSS_SOFTWARE_RECEIVERS/POSTPROCESSING_SCILAB_RECEIVERS/GLONASS"


@pytest.fixture(scope="module")
def z():
    return TR.load()


def _replay(z, run, **over):
    st, fch, acq_freq, code_phase, skip, sums = TR.run_inputs(z, run)
    s = S.settings(1, **{**TR.scilab_settings(st), **over})
    return S.replay(sums, s, fch, code_phase, acq_freq, skip=skip)


@pytest.mark.parametrize("run", TR.RUNS)
def test_oracle_loop_replays_the_recorded_run(z, run):
    r = _replay(z, run)
    assert len(r["blksize"]) == 1500
    TR.check_against_record(z, run, r, r["blksize"])


@pytest.mark.parametrize("run", TR.RUNS)
def test_record_pins_the_unaided_code_nco(z, run):
    """The current tracking.sci (:367-370, carrier-aided codeFreq) does not
    reproduce the record, so the record decides the variant."""
    st = dict(zip(list(z["settings_names"]), z[f"{run}_settings"].tolist()))
    r = _replay(z, run, codeNcoVariant=0, GLONASS_zero_channel=1602e6)
    assert not np.array_equal(r["codeFreq"], z[f"{run}_codeFreq"])
    r = _replay(z, run, absSampleVariant=0)
    assert not np.array_equal(r["absoluteSample"], z[f"{run}_absoluteSample"])
    assert st["codeLength"] == 511


@pytest.mark.parametrize("run", TR.RUNS)
def test_recorded_pll_discriminator_is_atan_of_the_sums(z, run):
    """tracking.sci:341 on the recorded prompt sums (ulp-level: libm atan)."""
    want = z[f"{run}_pllDiscr"]
    got = np.arctan(z[f"{run}_Q_P"] / z[f"{run}_I_P"]) / (2.0 * np.pi)
    assert np.max(np.abs(got - want) / np.abs(want)) < 1e-15


def test_record_settings_against_the_restated_defaults(z):
    """The recorded L1 settings vs sgt_oracle.settings(1) (initSettings.sci now):
    the signal constants and the PLL/FLL bandwidths agree; the DLL was run with
    a wider correlator spacing and bandwidth than the current defaults."""
    st = dict(zip(list(z["settings_names"]), z["L1_settings"].tolist()))
    d = S.settings(1)
    for k in ("samplingFreq", "codeFreqBasis", "codeLength", "IF", "L1_IF_step",
              "dllDampingRatio", "pllNoiseBandwidth", "fllNoiseBandwidth", "fileType"):
        assert st[k] == d[k], k
    assert (st["dllCorrelatorSpacing"], d["dllCorrelatorSpacing"]) == (0.5, 0.05)
    assert (st["dllNoiseBandwidth"], d["dllNoiseBandwidth"]) == (2.0, 0.5)
    assert st["skipNumberOfBytes"] == 16e6 and st["msToProcess"] == 1500


@pytest.mark.skipif(not os.path.isdir(SCI), reason="reference tree not mounted")
@pytest.mark.parametrize("run", TR.RUNS)
def test_fixture_equals_a_fresh_decode(z, run):
    """The committed fixture is exactly what the reader decodes from the .dat."""
    d = scilab_save.load(os.path.join(SCI, run, "trackingResults.dat"))
    assert list(d) == ["trackResults", "settings", "acqResults", "channel"]
    tr = d["trackResults"][0]
    for k in ("absoluteSample", "codeFreq", "carrFreq", *TR.SUMS, "dllDiscr", "dllDiscrFilt",
              "pllDiscr", "pllDiscrFilt"):
        np.testing.assert_array_equal(np.asarray(tr[k]).ravel(), z[f"{run}_{k}"])
    assert tr["status"] == "T" and float(tr["SVN"][0, 0]) == 4.0
    assert d["trackResults"][1]["SVN"].size == 0        # channel 2 never acquired


def test_reader_name_codes():
    """Scilab character codes with the upper-case borrow (oracle/scilab_save.py)."""
    def pack(codes):
        codes = codes + [40] * (24 - len(codes))
        words = []
        for i in range(0, 24, 4):
            c = codes[i:i + 4]
            words.append((c[0] + 256 * c[1] + 65536 * c[2] + 16777216 * c[3]) & 0xFFFFFFFF)
        return np.array(words, dtype="<u4").tobytes()
    # t r a c k R e s u l t s
    codes = [29, 27, 10, 12, 20, -27, 14, 28, 30, 21, 29, 28]
    assert scilab_save._name(pack(codes)) == "trackResults"
    assert scilab_save._name(pack([-29, 1, 36, 13])) == "T1_d"
