"""GPU: several IF records per acquisition launch (gnsscorr_acq_set_records).

A search over R records laid end to end must give, for every record, exactly
what a separate acquisition.sci search of that record gives (the same fp64
arithmetic on the same unit; only the launch shape changes): results and rows
bit-identical to R single-record searches, for both compiled plans, both block
modes, coherent integration and packed IF; one record is also held to the fp64
oracle (tests/test_acq_gpu.py check_rows).
"""
import numpy as np
import pytest

import acq_oracle as A
from test_acq_gpu import check_rows

pytestmark = pytest.mark.gpu


def _records(gpu, fs, n, nb, R, seed):
    out = []
    for r in range(R):
        sigs = [dict(system=0, prn=3 + 5 * r, code_phase=100.0 + 211.0 * r,
                     doppler=-2500.0 + 1500.0 * r, cn0=48.0),
                dict(system=0, prn=19, code_phase=700.5 - 50 * r, doppler=1000.0, cn0=46.0)]
        out.append(gpu.ifgen(nb * n, sigs, fs=fs, seed=seed + r))
    return out


@pytest.mark.parametrize("fs,n", [(16.368e6, 16368), (16.0e6, 16000)])
@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_records_equal_single_searches(gpu, fs, n, mode):
    R, nb = 3, 2 if mode == "best" else 4
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    recs = _records(gpu, fs, n, nb, R, 0x5EED0050)
    prns = [3, 8, 13, 19]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    freqs = A.gps_bins(2.42e6, 8, 1)
    gf = np.tile(np.arange(len(freqs)), (len(prns), 1))
    single = gpu.AcqCtx(fs, n, max_freqs=64, max_blocks=nb, max_codes=8)
    single.set_codes(codes)
    ref = [single.search(x, nb, freqs, np.arange(len(prns)), gf, mode=m) for x in recs]
    batch = gpu.AcqCtx(fs, n, max_freqs=64, max_blocks=nb * R, max_codes=8)
    batch.set_codes(codes)
    batch.set_records(R)
    res, rows = batch.search(np.concatenate(recs), nb, freqs, np.arange(len(prns)), gf, mode=m)
    assert res.shape == (R, len(prns)) and rows.shape == (R, len(prns), len(freqs))
    for r in range(R):
        assert res[r].tobytes() == ref[r][0].tobytes(), f"record {r} results"
        assert rows[r].tobytes() == ref[r][1].tobytes(), f"record {r} rows"
    # the planted PRN of every record is found in its own record
    for r in range(R):
        assert res[r][[3, 8, 13, 19].index(3 + 5 * r)]["metric"] > 2.5


@pytest.mark.parametrize("fs,n,chunk_mb", [(38.192e6, 38192, "2"), (38.192e6, 38192, "0"),
                                           (5.0e6, 5000, "0")])
@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_generic_records_equal_single_searches(gpu, fs, n, chunk_mb, mode, monkeypatch):
    """Records on the generic engine (the four-step plan at 38 192, with 2 MiB chunks so
    the records' units cross chunk and lane boundaries; the mixed-radix passes at 5000):
    every record bit-identical to its own single-record search."""
    if chunk_mb != "0":
        monkeypatch.setenv("GNSSCORR_ACQ_GCHUNK_MB", chunk_mb)
    R, nb = 3, 2 if mode == "best" else 4
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    recs = _records(gpu, fs, n, nb, R, 0x5EED0058)
    prns = [3, 8, 13, 19]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    freqs = A.gps_bins(2.42e6, 8, 1)
    gf = np.tile(np.arange(len(freqs)), (len(prns), 1))
    single = gpu.AcqCtx(fs, n, max_freqs=64, max_blocks=nb, max_codes=8)
    single.set_codes(codes)
    ref = [single.search(x, nb, freqs, np.arange(len(prns)), gf, mode=m) for x in recs]
    batch = gpu.AcqCtx(fs, n, max_freqs=64, max_blocks=nb * R, max_codes=8)
    batch.set_codes(codes)
    batch.set_records(R)
    res, rows = batch.search(np.concatenate(recs), nb, freqs, np.arange(len(prns)), gf, mode=m)
    assert res.shape == (R, len(prns)) and rows.shape == (R, len(prns), len(freqs))
    for r in range(R):
        assert res[r].tobytes() == ref[r][0].tobytes(), f"record {r} results"
        assert rows[r].tobytes() == ref[r][1].tobytes(), f"record {r} rows"
    # (the single-record searches themselves are held to the oracle in
    # test_acq_generic_gpu.py; the scenes here are the compiled-plan test's, weaker at
    # these rates, so no detection threshold is asserted)


def test_records_vs_oracle(gpu):
    fs, n, nb, R = 16.368e6, 16368, 2, 2
    recs = _records(gpu, fs, n, nb, R, 0x5EED0060)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (8, 19)])
    freqs = A.gps_bins(2.42e6, 6, 1)
    gf = np.tile(np.arange(len(freqs)), (2, 1))
    ctx = gpu.AcqCtx(fs, n, max_freqs=32, max_blocks=nb * R, max_codes=2)
    ctx.set_codes(codes)
    ctx.set_records(R)
    res, rows = ctx.search(np.concatenate(recs), nb, freqs, np.arange(2), gf)
    ref, ref_rows = A.acquire(recs[1], fs, codes, freqs, gf, n_blocks=nb, return_rows=True)
    check_rows(res[1], rows[1], ref, ref_rows, True, label="records[1]")


def test_records_coherent_packed_and_dev(gpu):
    """5-ms coherent blocks from packed bytes, through the device-resident API."""
    fs, n, coh, nb, R = 16.368e6, 16368, 5, 2, 2
    recs = _records(gpu, fs, n, coh * nb, R, 0x5EED0070)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (3, 8, 19)])
    freqs = 2.42e6 + 100.0 * np.arange(-8, 9)
    gf = np.tile(np.arange(len(freqs)), (3, 1)).astype(np.int32)
    gcode = np.arange(3, dtype=np.int32)
    iq = gpu.iq_flags(True, True)
    single = gpu.AcqCtx(fs, n, max_freqs=32, max_blocks=coh * nb, max_codes=4)
    single.set_codes(codes)
    single.set_coherent(coh)
    ref = [single.search(gpu.pack2(x), nb, freqs, gcode, gf, iq=iq) for x in recs]
    ctx = gpu.AcqCtx(fs, n, max_freqs=32, max_blocks=coh * nb * R, max_codes=4)
    ctx.set_codes(codes)
    ctx.set_coherent(coh)
    ctx.set_records(R)
    d_if = gpu.DevBuf.from_array(gpu.pack2(np.concatenate(recs)))
    d_freqs, d_gc, d_gf = (gpu.DevBuf.from_array(a) for a in (freqs, gcode, gf))
    d_rows = gpu.DevBuf(R * 3 * len(freqs) * gpu.ACQ_ROW.itemsize)
    d_res = gpu.DevBuf(R * 3 * gpu.ACQ_RESULT.itemsize)
    ctx.spectra_dev(d_if.ptr, nb, len(freqs), d_freqs.ptr, iq=iq)
    ctx.correlate_dev(nb, d_freqs.ptr, 3, len(freqs), d_gc.ptr, d_gf.ptr)
    ctx.select_dev(3, len(freqs), d_freqs.ptr, d_gf.ptr, d_rows.ptr, d_res.ptr)
    ctx.sync()
    res = d_res.download(gpu.ACQ_RESULT).reshape(R, 3)
    rows = d_rows.download(gpu.ACQ_ROW).reshape(R, 3, len(freqs))
    for r in range(R):
        assert res[r].tobytes() == ref[r][0].tobytes()
        assert rows[r].tobytes() == ref[r][1].reshape(3, -1).tobytes()


def test_records_refused(gpu):
    with pytest.raises(gpu.GnssCorrError):      # fp32 fast path: one record
        gpu.AcqCtx(16.368e6, 16368, max_blocks=4, precision=gpu.ACQ_F32).set_records(2)
    with pytest.raises(gpu.GnssCorrError):      # Bluestein engine (N = 4111, prime): one record
        gpu.AcqCtx(4.111e6, 4111, max_blocks=4).set_records(2)
    ctx = gpu.AcqCtx(16.368e6, 16368, max_freqs=4, max_blocks=4, max_codes=1)
    ctx.set_codes(A.make_ca_table_row(1, 16.368e6)[None])
    ctx.set_records(3)
    with pytest.raises(gpu.GnssCorrError):      # 3 records x 2 blocks > max_blocks
        ctx.search(np.zeros(6 * 2 * 16368, np.int8), 2, [2.42e6], [0], [[0]])
