"""CPU: the GPS-SDR int16 acquisition oracle (oracle/sdr_acq.c) pinned against
the reference primitives compiled from their own sources (-DNO_SIMD,
oracle/_ref/libsdr_ref.so) and against the committed fixtures
(tests/golden/sdr_*.npz, made by tests/golden/make_sdr_golden.py), plus the
product's host tables (PRN_Codes, sine_gen) against the same fixtures.

Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER objects/fft.cpp,
simd/x86.cpp, accessories/misc.cpp, accessories/gen_fft_codes.m,
objects/acquisition.cpp:191-301.
"""
import os

import numpy as np
import pytest

import sdr_oracle as S

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
need_ref = pytest.mark.skipif(not S.have_ref(), reason="reference build (oracle/_ref) absent")


@pytest.fixture(scope="module")
def o(oracle):
    return S.OracleSDR()


def test_prn_codes_golden(o, gc):
    g = np.load(os.path.join(GOLD, "sdr_prn_codes.npz"))["prn_codes"]
    assert g.shape == (51, 2048, 2)
    assert (o.prn_codes() == g).all()            # oracle restatement of gen_fft_codes.m
    assert (gc.sdr_prn_codes() == g).all()       # the product's table
    # 9-bit scaling: the largest magnitude over all 51 codes is 512
    assert np.abs(g.astype(np.float64)).max() <= 512


def test_fft_golden(o):
    f = np.load(os.path.join(GOLD, "sdr_fft.npz"))
    for x, fw, iv in zip(f["x"], f["fwd_r1"], f["inv_r2"]):
        assert (o.fft(x, False, S.R1) == fw).all()
        assert (o.fft(x, True, S.R2) == iv).all()


def test_acq_strong_golden(o):
    f = np.load(os.path.join(GOLD, "sdr_acq.npz"))
    codes = np.load(os.path.join(GOLD, "sdr_prn_codes.npz"))["prn_codes"]
    for b, res, nar in zip(f["buffers"], f["res"], f["res_narrow"]):
        got = o.acq_strong(b, codes, f["svs"], fif=float(f["fif"]))
        assert (got == res).all()
        got = o.acq_strong(b, codes, f["svs"], -3000, 5000, fif=float(f["fif"]))
        assert (got == nar).all()


def test_planted_signals_found(o):
    f = np.load(os.path.join(GOLD, "sdr_acq.npz"))
    r = f["res"][0]
    # scene 0: PRN 5 at 300 chips / +2250 Hz -> code_phase 2048 - 2*(1023-300)... as sampled
    assert r[4]["doppler"] == 2250 and abs(r[4]["code_phase"] - 600) <= 1
    assert r[4]["magnitude"] > 5 * np.median(r["magnitude"])


@need_ref
def test_oracle_matches_reference_build(o):
    ref = S.RefSDR()
    for f in (-38400.0, -38650.0, -38900.0, -39150.0, 1000.5, 0.0):
        assert (o.sine_gen(f) == ref.sine_gen(f)).all()
    rng = np.random.default_rng(5)
    for amp in (3, 1000, 32767):
        x = rng.integers(-amp, amp + 1, (2048, 2)).astype(np.int16)
        y = rng.integers(-amp, amp + 1, (2048, 2)).astype(np.int16)
        for inv in (False, True):
            for sc in (S.R1, S.R2, np.ones(16, np.int32)):
                assert (o.fft(x, inv, sc) == ref.fft(x, inv, sc)).all()
        for sh in (10, 14):
            assert (o.cmulsc(x, y, sh) == ref.cmulsc(x, y, sh)).all()
        assert o.cmag_max(x) == ref.cmag_max(x)
    assert (o.prn_codes() == ref.prn_codes()).all()
    buf = S.make_buffer([dict(prn=9, code_phase=123.0, doppler=-6400.0, amp=1.0)], seed=77)
    svs = [8, 0, 20]
    assert (o.acq_strong(buf, ref.prn_codes(), svs) == ref.acq_strong(buf, svs)).all()


def test_saturating_cmulsc_differs_only_on_overflow(o):
    x = np.array([[32767, 32767], [-32768, 5], [100, -100]], np.int16)
    y = np.array([[32767, -32767], [-32768, 0], [3, 4]], np.int16)
    w, s = o.cmulsc(x, y, 1), o.cmulsc(x, y, 1, saturate=True)
    assert (w[2] == s[2]).all()
    assert s[0, 0] == 32767 or s[0, 1] in (32767, -32768)
    assert not (w[:2] == s[:2]).all()


# ---------------------------------------------------------------- tracking correlator
@pytest.fixture(scope="module")
def oc(oracle):
    return S.OracleSdrCorr()


def test_corr_tables_and_accum_golden(oc):
    import hashlib
    g = np.load(os.path.join(GOLD, "sdr_corr.npz"))
    assert hashlib.sha256(oc.carrier.tobytes()).hexdigest() == str(g["carrier_sha256"])
    for sv in range(32):
        assert (oc.code_gen(sv) == g["chips"][sv]).all()
        # SamplePRN row lcv=25 (phase 0) is the chip sequence at 2 samples/chip-ish
        row = oc.code[sv, 25]
        assert set(np.unique(row)) <= {-1, 1}
    for job, d, exp in zip(g["jobs"], g["data"], g["expected"]):
        j = dict(packet=job[0], data_off=job[1], samps=job[2], sv=job[3], sbin=job[4],
                 soff=job[5], cbin=job[6:9], coff=job[9:12])
        c = oc.accum(d, j)
        got = np.array([c["i"][0], c["q"][0], c["i"][1], c["q"][1], c["i"][2], c["q"][2]])
        assert (got == exp).all()


@need_ref
def test_corr_primitives_match_reference_build(oc):
    ref = S.RefSDR()
    for sv in range(32):
        assert (oc.code_gen(sv) == ref.code_gen(sv)).all()
    for k in (-1500, -1, 0, 1, 777, 1500):
        assert (oc.carrier[k + 1500] == ref.sine_gen(np.float32(-38400.0) - np.float32(k) *
                                                     np.float32(10.0), n=4096)).all()


def test_correlator_flow_tracks_a_planted_signal(oc):
    """Correlator::Correlate + the test loop on 300 packets: dumps once per code
    period, the prompt arm dominates, epoch counters advance."""
    sig = dict(prn=7, code_phase=200.0, doppler=1500.0, amp=4.0)
    K = 300
    buf = S.make_buffer([sig], n=K * 2048, seed=4, amp_noise=2.0)
    # acquisition-style start: code phase in samples of the C/A start, doppler
    cp_samples = int(round((1023 - 200.0) * 2))
    st = np.zeros(1, S.CHAN)
    st[0] = oc.init_chan(6, cp_samples, 1500)
    corr = np.zeros(1, S.CORR)
    counts = []
    for k in range(K):
        oc.correlate(buf[k * 2048:(k + 1) * 2048], st, corr)
        counts.append(int(st[0]["count"]))
    assert 295 <= counts[-1] <= 302
    assert st[0]["active"] == 1


# ---- sample front end (SDR/objects/gps_source.cpp:684-767, :933-943; misc.cpp:174-197)
def test_downsample_oracle_golden():
    f = np.load(os.path.join(GOLD, "sdr_frontend.npz"))
    o = S.OracleSDR()
    for src, out, (fs, n, k) in zip(f["src"], f["out"], f["rates"]):
        n, k = int(n), int(k)
        got = o.downsample(src[:n], 2.048e6, fs)
        assert got.shape[0] == k and np.array_equal(got, out[:k]), fs


def test_downsample_count_closed_form():
    import gnsscorr
    o = S.OracleSDR()
    rng = np.random.default_rng(2)
    for fs in (2.1e6, 4.0e6, 4.096e6, 5.0e6, 8.0e6, 16.368e6):
        for n in (1, 2, 7, 4000, 4096, 16368):
            src = rng.integers(-5, 5, (n, 2)).astype(np.int16)
            assert gnsscorr.SdrFeCtx.downsample_count(n, 2.048e6, fs) == \
                o.downsample(src, 2.048e6, fs).shape[0], (fs, n)


@pytest.mark.skipif(not S.have_ref(), reason="reference build needs /root/reference")
def test_downsample_oracle_vs_reference():
    o, r = S.OracleSDR(), S.RefSDR()
    rng = np.random.default_rng(4)
    for fs in (3.0e6, 4.0e6, 6.5536e6, 16.0e6):
        src = rng.integers(-30000, 30000, (int(fs / 1000) * 2, 2)).astype(np.int16)
        assert np.array_equal(o.downsample(src, 2.048e6, fs), r.downsample(src, 2.048e6, fs))


def test_gn3s_oracle_vs_product_table():
    """The oracle's double-product path equals the library's int16 product table
    indexed by (2-bit code, phase >> 22); resample picks floor((i+1)*4000/2048)."""
    import gnsscorr
    o = S.OracleSDR()
    prod = gnsscorr.gn3s_products()
    rng = np.random.default_rng(7)
    raw = rng.integers(0, 256, 2 * 20000, dtype=np.uint8)
    ph0 = 987654321
    out, ph = o.gn3s(raw, ph0)
    n = np.arange(2 * 20000, dtype=np.uint64)
    phases = ((ph0 + n * 2557223528) % (1 << 32)) >> 22
    mixed = prod[raw & 3, phases.astype(np.int64)].reshape(2, 20000, 2)
    idx = ((np.arange(10240) + 1) * 4000) // 2048
    for b in range(2):
        ok = idx < 20000
        assert np.array_equal(out.reshape(2, 10240, 2)[b][ok], mixed[b][idx[ok]])
        assert (out.reshape(2, 10240, 2)[b][~ok] == 0).all()
    assert ph == (ph0 + 2 * 20000 * 2557223528) % (1 << 32)


# ---- medium / weak acquisition (acquisition.cpp:191-236, 309-570) ---------------
def _mw_session_oracle(o, codes, buf, fif):
    """The golden's request sequence on the C restatement's row store."""
    rows = o.new_rows()
    o.prep_rows(rows, buf, 10, fif)
    med0 = o.acq_search("medium", rows, codes, np.arange(32))
    o.prep_rows(rows, buf, 310, fif)
    return rows, med0


def test_acq_medium_weak_golden(o):
    f = np.load(os.path.join(GOLD, "sdr_acq_mw.npz"))
    codes = np.load(os.path.join(GOLD, "sdr_prn_codes.npz"))["prn_codes"]
    buf = f["buffer"].astype(np.int16)
    rows, med0 = _mw_session_oracle(o, codes, buf, float(f["fif"]))
    assert (med0 == f["medium_fresh"]).all()
    assert (o.acq_search("weak", rows, codes, f["weak_svs"], -5000, 5000) == f["weak"]).all()
    o.prep_rows(rows, buf, 10, float(f["fif"]))
    assert (o.acq_search("medium", rows, codes, np.arange(32), -7000, 3000) ==
            f["medium_after_weak"]).all()
    # the planted signals: PRN 5 strong enough for both, PRN 26 only non-coherently
    w = {int(r["sv"]): r for r in f["weak"]}
    assert w[4]["doppler"] == 2350 and w[25]["magnitude"] > 3 * w[9]["magnitude"]


def test_weak_code_doppler_shift(o):
    # acquisition.cpp:483-489 at the extremes of the +-15 kHz search
    assert o.weak_shift(0, 14, 3) == 0
    assert o.weak_shift(14, 14, 3) == int(np.floor(14 * .02 * 2048000 * 14750.0 / 1.57542e9))
    assert o.weak_shift(14, -15, 0) == int(np.floor(14 * .02 * 2048000 * -15000.0 / 1.57542e9))
    assert o.weak_shift(14, -15, 0) < 0


@need_ref
def test_medium_weak_oracle_matches_reference_build(o):
    ref = S.RefSDR()
    codes = ref.prn_codes()
    rng = np.random.default_rng(8)
    for amp, sat_range in ((2.0, 3), (90.0, 5)):
        buf = S.make_long_buffer([dict(prn=11, code_phase=500.5, doppler=-1250.0, amp=amp / 4)],
                                 310, seed=int(rng.integers(1 << 20)), amp_noise=amp)
        sess = S.RefAcqSession(ref)
        rows = o.new_rows()
        sess.prep(buf, 310)
        o.prep_rows(rows, buf, 310)
        assert (o.acq_search("weak", rows, codes, [10, 3], -2000, 0) ==
                sess.search("weak", [10, 3], -2000, 0)).all()
        sess.prep(buf, 10)
        o.prep_rows(rows, buf, 10)
        assert (o.acq_search("medium", rows, codes, [10, 3, 31], -sat_range * 1000, 1999) ==
                sess.search("medium", [10, 3, 31], -sat_range * 1000, 1999)).all()
    # full-scale int16 input: the FFT ranks, the >> 16 and cmag wrap identically
    big = rng.integers(-32768, 32768, (310 * 2048, 2)).astype(np.int16)
    sess = S.RefAcqSession(ref)
    rows = o.new_rows()
    sess.prep(big, 10)
    o.prep_rows(rows, big, 10)
    assert (o.acq_search("medium", rows, codes, [0, 7], -1000, 1000) ==
            sess.search("medium", [0, 7], -1000, 1000)).all()
