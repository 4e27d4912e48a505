"""GPU parity at the Scilab receivers' own settings: 16 Msps, samplesPerCode 16000.

Reference settings:
  GPS      SCI/GPS/L1/initSettings.sci:68-87      IF 2.42 MHz, fs 16 MHz,
           acqSearchBand 14 kHz, acqCohIntegration 4 -> 113 bins at 125 Hz
  GLONASS  SCI/GLONASS/L1/initSettings.sci:69-96  IF 1 MHz, fs 16 MHz,
           acqSearchBand 12 kHz, acqCohIntegration 5 -> 121 bins at 100 Hz
samplesPerCode = round(fs / (codeFreqBasis / codeLength)) = 16000
(acquisition.sci:47-48), samplesPerCodeChip = round(fs / codeFreqBasis) = 16 (GPS) /
31 (GLONASS).  The fp64 path (16000 = 40 x 40 x 10 Cooley-Tukey plan) is held to the
north_star 1e-6 relative tolerance with exact decisions, against the literal
coh*N-point fp64 oracle (oracle/acq_oracle.py).
"""
import numpy as np
import pytest

import acq_oracle as A
from test_acq_gpu import check_rows

pytestmark = pytest.mark.gpu
FS = 16.0e6
N = 16000


def test_gps_default_settings_coh4(gpu):
    coh, band = 4, 14
    ctx = gpu.AcqCtx(FS, N, max_freqs=256, max_blocks=2 * coh, max_codes=32)
    prns = [4, 17, 30]
    codes = np.stack([A.make_ca_table_row(p, FS) for p in prns])
    assert codes.shape[1] == N
    ctx.set_codes(codes)
    ctx.set_coherent(coh)
    sigs = [dict(system=0, prn=4, code_phase=333.3, doppler=-2875.0, cn0=40.0, data_bits=1),
            dict(system=0, prn=30, code_phase=12.0, doppler=5125.0, cn0=42.0, data_bits=1)]
    IF = gpu.ifgen(2 * coh * N, sigs, fs=FS, seed=0x5EED0016)
    freqs = A.gps_bins(2.42e6, band, coh)                # 113 bins @ 125 Hz
    assert len(freqs) == 113
    gf = np.tile(np.arange(len(freqs)), (3, 1))
    res, rows = ctx.search(IF, 2, freqs, np.arange(3), gf, spc=16)
    ref, ref_rows = A.acquire(IF, FS, codes, freqs, gf, spc=16, coh=coh, return_rows=True)
    check_rows(res, rows, ref, ref_rows, True, label="gps-16M-coh4")
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5


def test_glonass_default_settings_coh5(gpu):
    coh, band = 5, 12
    ctx = gpu.AcqCtx(FS, N, max_freqs=2048, max_blocks=2 * coh, max_codes=1)
    code = A.make_st_table_row(FS)[None]
    assert code.shape[1] == N
    ctx.set_codes(code)
    ctx.set_coherent(coh)
    sigs = [dict(system=1, fch=-2, code_phase=140.0, doppler=1650.0, cn0=41.0),
            dict(system=1, fch=3, code_phase=410.0, doppler=-2300.0, cn0=43.0)]
    IF = gpu.ifgen(2 * coh * N, sigs, fs=FS, if_glo=1.0e6, seed=0x5EED0017)
    fchs = [-2, 0, 3]
    per = A.gps_bins(0.0, band, coh)                     # 121 bins @ 100 Hz
    assert len(per) == 121
    freqs = np.concatenate([1.0e6 + k * 0.5625e6 + per for k in fchs])
    gf = np.arange(len(fchs) * len(per)).reshape(len(fchs), len(per))
    gcode = np.zeros(len(fchs), np.int32)
    res, rows = ctx.search(IF, 2, freqs, gcode, gf, spc=31)
    ref, ref_rows = A.acquire(IF, FS, code, freqs, gf, group_code=gcode, spc=31, coh=coh,
                              return_rows=True)
    check_rows(res, rows, ref, ref_rows, True, label="glonass-16M-coh5")
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5


def test_power_row_16000(gpu):
    ctx = gpu.AcqCtx(FS, N, max_freqs=8, max_blocks=2, max_codes=2)
    codes = np.stack([A.make_ca_table_row(p, FS) for p in (9, 22)])
    ctx.set_codes(codes)
    IF = gpu.ifgen(2 * N, [dict(system=0, prn=22, code_phase=700.25, doppler=-1500.0,
                                cn0=48.0)], fs=FS, seed=12)
    for code, freq, blk in [(1, 2.42e6 - 1500.0, 0), (0, 2.42e6 + 3333.0, 1)]:
        got = ctx.power_row(IF, 2, blk, freq, code)
        ref = A.power_rows(IF, FS, codes[code], freq)[blk]
        err = np.abs(got - ref).max() / ref.max()
        print(f"[power row 16000] code {code} freq {freq}: {err:.3e}")
        assert err < 1e-6
        assert np.argmax(got) == np.argmax(ref)


def test_noncoherent_16000(gpu):
    ctx = gpu.AcqCtx(FS, N, max_freqs=16, max_blocks=10, max_codes=2)
    codes = np.stack([A.make_ca_table_row(p, FS) for p in (11, 2)])
    ctx.set_codes(codes)
    IF = gpu.ifgen(10 * N, [dict(system=0, prn=11, code_phase=50.0, doppler=900.0,
                                 cn0=39.0)], fs=FS, seed=13)
    freqs = A.gps_bins(2.42e6, 4)
    gf = np.tile(np.arange(len(freqs)), (2, 1))
    res, rows = ctx.search(IF, 10, freqs, [0, 1], gf, mode=gpu.ACQ_NONCOHERENT)
    ref, ref_rows = A.acquire(IF, FS, codes, freqs, gf, n_blocks=10, noncoherent=True,
                              return_rows=True)
    for rr in ref_rows:
        for r in rr:
            r["block"] = -1
    check_rows(res, rows, ref, ref_rows, True, label="noncoherent-16000")
