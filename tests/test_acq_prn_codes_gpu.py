"""gnsscorr_acq_set_prn_codes: the code replicas generated on the device from code
ids (acquisition.sci:91-95: caCodesTable = makeCaTable(settings), then
conj(fft(caCodesTable(PRN,:))) inside every search) against host replicas
(gnsscorr_ca_code / gnsscorr_st_code + gnsscorr_sample_code, themselves pinned to
the ICD octal KATs and the numpy restatement in tests/test_codes_host.py) uploaded
with gnsscorr_acq_set_codes.  The replicas are the same bytes, so every search
statistic must be bit-identical; covers the compiled fp64 plans (16.368 and 16
Msps), the generic engine (5 and 38.192 Msps), the fp32 path and the GLONASS ST id."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _host_codes(gc, ids, fs, n):
    rows = []
    for p in ids:
        if p == gc.CODE_GLO_ST:
            rows.append(gc.sample_code(gc.st_code(), 0.511e6, fs, n))
        else:
            rows.append(gc.sample_code(gc.ca_code(int(p)), 1.023e6, fs, n))
    return np.stack(rows)


@pytest.mark.parametrize("fs,prec", [(16.368e6, "f64"), (16.0e6, "f64"), (5.0e6, "f64"),
                                     (38.192e6, "f64"), (16.368e6, "f32")])
def test_device_codes_equal_host_codes(gpu, fs, prec):
    n = int(round(fs / 1000.0))
    ids = np.array([3, 17, gpu.CODE_GLO_ST, 32, 1], np.int32)
    sigs = [dict(system=0, prn=17, code_phase=300.25, doppler=1500.0, cn0=50.0),
            dict(system=1, prn=0, code_phase=100.5, doppler=-500.0, cn0=50.0, fch=0)]
    IF = gpu.ifgen(2 * n, sigs, fs=fs, seed=0x5EED0040)
    freqs = 2.42e6 + 500.0 * np.arange(-6, 7)
    gf = np.tile(np.arange(len(freqs)), (len(ids), 1))
    kw = dict(precision=gpu.ACQ_F32 if prec == "f32" else gpu.ACQ_F64)
    out = []
    for dev in (False, True):
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=2, max_codes=len(ids), **kw)
        if dev:
            ctx.set_prn_codes(ids)
        else:
            ctx.set_codes(_host_codes(gpu, ids, fs, n))
        out.append(ctx.search(IF, 2, freqs, np.arange(len(ids)), gf, spc=max(1, n // 1023)))
    (r0, w0), (r1, w1) = out
    assert r0.tobytes() == r1.tobytes()
    assert w0.tobytes() == w1.tobytes()
    assert r0[1]["metric"] > 2.5   # PRN 17 is planted


def test_prn_codes_rejects_bad_ids(gpu):
    ctx = gpu.AcqCtx(16.368e6, 16368, max_freqs=4, max_blocks=2, max_codes=2)
    for bad in ([33, 1], [-1], [1, 2, 3]):
        with pytest.raises(gpu.GnssCorrError):
            ctx.set_prn_codes(bad)
