"""GPU parity: multi-ms coherent acquisition (settings.acqCohIntegration, the
GLONASS receiver's default 5 ms), SURVEY 8(f) rank 3.

Reference: POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/acquisition.sci:52-72,
100-135 (coh*N-sample blocks, one phase ramp, code repmat'ed coh times,
coh*N-point FFTs, rows = first code period).  The oracle
(oracle/acq_oracle.py, coh=) runs that literally in fp64 with 81 840-point
transforms; the GPU folds the wiped-off block into one code period first (the
coh*N spectrum is zero off multiples of coh, see acq.hip).  Tolerances as in
test_acq_gpu.py: fp64 -- 1e-6 relative everywhere, decisions exact; fp32 --
powers 2e-5 of the row max, peaks 1e-4, decisions exact when the oracle's
winner is clear.
"""
import numpy as np
import pytest

import acq_oracle as A
from test_acq_gpu import check_rows

pytestmark = pytest.mark.gpu
FS, N, COH = 16.368e6, 16368, 5


def _glo(fch, cp, dop, cn0):
    return dict(system=1, fch=fch, code_phase=cp, doppler=dop, cn0=cn0)


@pytest.fixture(scope="module", params=["f64", "f32"])
def ctx(request, gpu):
    prec = gpu.ACQ_F64 if request.param == "f64" else gpu.ACQ_F32
    c = gpu.AcqCtx(FS, N, max_freqs=256, max_blocks=2 * COH, max_codes=4, precision=prec)
    c.set_codes(A.make_st_table_row(FS)[None])
    c.set_coherent(COH)
    return c


def _literal_row(IF, code, freq, blk):
    sig = A._signal(IF, True)
    L = COH * N
    pp = np.arange(L) * 2 * np.pi / FS
    X = np.fft.fft(np.exp(1j * freq * pp) * sig[blk * L:(blk + 1) * L])
    cf = np.conj(np.fft.fft(np.tile(code.astype(np.float64), COH)))
    return (np.abs(np.fft.ifft(X * cf)) ** 2)[:N]


def test_power_rows_5ms(gpu, ctx):
    IF = gpu.ifgen(2 * COH * N, [_glo(2, 40.0, 350.0, 42.0)], fs=FS, if_glo=1e6, seed=8)
    code = A.make_st_table_row(FS)
    f0 = 1e6 + 2 * 0.5625e6
    for freq, blk in [(f0 + 300.0, 0), (f0 + 400.0, 1), (f0 - 1200.0, 0)]:
        got = ctx.power_row(IF, 2, blk, freq, 0)
        ref = _literal_row(IF, code, freq, blk)
        err = np.abs(got - ref).max() / ref.max()
        assert err < (1e-6 if ctx.precision == 0 else 2e-5), (freq, blk, err)
        assert np.argmax(got) == np.argmax(ref)


def test_glonass_fch_search_5ms(gpu, ctx):
    """3 FCH x 11 bins (1 kHz band at 1000/(2*5) = 100 Hz): a 39 dB-Hz signal (metric
    1.7 at 1 ms, above 4.5 at 5 ms in the oracle) and a 42 dB-Hz one."""
    IF = gpu.ifgen(2 * COH * N, [_glo(-4, 300.0, -250.0, 42.0), _glo(5, 77.0, 120.0, 39.0)],
                   fs=FS, if_glo=1e6, seed=21)
    fchs = [-4, 0, 5]
    band_khz = 1.0
    nb = int(round(band_khz * 2 * COH)) + 1
    freqs, gf = [], []
    for g, k in enumerate(fchs):   # acquisition.sci:105-108 bin grid per FCH
        c0 = 1e6 + k * 0.5625e6
        fb = c0 - (band_khz / 2) * 1000 + (1000 / (2 * COH)) * np.arange(nb)
        gf.append(np.arange(len(freqs), len(freqs) + nb))
        freqs.extend(fb)
    freqs, gf = np.array(freqs), np.array(gf)
    code = A.make_st_table_row(FS)[None]
    res, rows = ctx.search(IF, 2, freqs, np.zeros(3, np.int32), gf, spc=32)
    ref, ref_rows = A.acquire(IF, FS, code, freqs, gf, group_code=np.zeros(3, int), spc=32,
                              coh=COH, return_rows=True)
    check_rows(res, rows, ref, ref_rows, ctx.precision == 0, label="glonass-5ms")
    assert res[0]["metric"] > 3 and res[2]["metric"] > 3 and res[1]["metric"] < 3


def test_set_coherent_bounds(gpu, ctx):
    with pytest.raises(gpu.GnssCorrError):
        ctx.set_coherent(0)
    with pytest.raises(gpu.GnssCorrError):
        ctx.set_coherent(2 * COH + 1)
    ctx.set_coherent(COH + 1)          # 2 blocks x 6 ms no longer fit max_blocks = 10
    try:
        with pytest.raises(gpu.GnssCorrError):
            ctx.search(np.zeros(2 * 6 * N * 2, np.int8), 2, np.array([1e6]),
                       np.zeros(1, np.int32), np.zeros((1, 1), np.int32), spc=32)
    finally:
        ctx.set_coherent(COH)
