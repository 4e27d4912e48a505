"""GPU parity: GPS-SDR sample front end (sdr_frontend.hip), bit-exact.

Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/
objects/gps_source.cpp:684-767 (Read_GN3S), :933-943 (Resample_GN3S),
accessories/misc.cpp:174-197 (downsample).  Checked against the C restatement
(oracle/sdr_frontend.c) and the reference build's downsample known answers
(tests/golden/sdr_frontend.npz); the raw-bytes -> front end -> strong
acquisition chain is checked end to end against the oracle chain.
"""
import os

import numpy as np
import pytest

import sdr_oracle as S

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("packed", [False, True])
def test_gn3s_vs_oracle(gpu, oracle, packed):
    o = S.OracleSDR()
    rng = np.random.default_rng(3 + packed)
    raw = rng.integers(0, 256, 6 * 20000, dtype=np.uint8)
    phase0 = int(rng.integers(0, 1 << 32))
    want, wph = o.gn3s(raw & 3 if packed else raw, phase0)
    fe = gpu.SdrFeCtx()
    data = gpu.pack_2bit(raw) if packed else raw
    got, ph = fe.gn3s(data, packed=packed, phase=phase0)
    assert ph == wph
    assert np.array_equal(got, want)
    assert (got.reshape(6, 10240, 2)[:, -1] == 0).all()    # the stale buff[20000] read
    # two calls continue the NCO exactly like one
    per = 20000 // 4 if packed else 20000
    g1, p1 = fe.gn3s(data[:2 * per], packed=packed, phase=phase0)
    g2, p2 = fe.gn3s(data[2 * per:], packed=packed, phase=p1)
    assert p2 == wph and np.array_equal(np.concatenate([g1, g2]), want)


def test_gn3s_dev_large(gpu, oracle):
    """400 blocks (2 s of samples) on the device, packed input, spot-checked blocks."""
    o = S.OracleSDR()
    rng = np.random.default_rng(11)
    nb = 400
    raw = rng.integers(0, 4, nb * 20000, dtype=np.uint8)
    fe = gpu.SdrFeCtx()
    d_in = gpu.DevBuf.from_array(gpu.pack_2bit(raw))
    d_out = gpu.DevBuf(nb * 10240 * 4)
    ph = fe.gn3s_dev(d_in.ptr, True, nb, 12345, d_out.ptr)
    fe.sync()
    got = d_out.download(np.int16).reshape(nb, 10240, 2)
    _, want_ph = o.gn3s(raw[:20000], 12345)
    ph_k = 12345
    for k in (0, 1, 199, 399):
        ph_k = (12345 + k * 20000 * 2557223528) % (1 << 32)
        want, _ = o.gn3s(raw[k * 20000:(k + 1) * 20000], ph_k)
        assert np.array_equal(got[k], want), k
    assert ph == (12345 + nb * 20000 * 2557223528) % (1 << 32)


def test_gn3s_dev_misaligned_out(gpu):
    """The kernel writes 16-byte stores: a misaligned d_out is refused (EINVAL),
    nothing is launched and the caller's phase is left unchanged."""
    fe = gpu.SdrFeCtx()
    d_in = gpu.DevBuf.from_array(np.zeros(20000 // 4, np.uint8))
    d_out = gpu.DevBuf(10240 * 4 + 16)
    with pytest.raises(gpu.GnssCorrError, match="16-byte aligned"):
        fe.gn3s_dev(d_in.ptr, True, 1, 7, d_out.ptr + 4)


def test_downsample_golden(gpu):
    f = np.load(os.path.join(GOLD, "sdr_frontend.npz"))
    fe = gpu.SdrFeCtx()
    for src, out, (fs, n, k) in zip(f["src"], f["out"], f["rates"]):
        n, k = int(n), int(k)
        assert fe.downsample_count(n, 2.048e6, fs) == k
        d_src = gpu.DevBuf.from_array(src[:n])
        d_dst = gpu.DevBuf(k * 4)
        assert fe.downsample_dev(d_src.ptr, n, 2.048e6, fs, d_dst.ptr) == k
        fe.sync()
        assert np.array_equal(d_dst.download(np.int16).reshape(k, 2), out[:k]), fs


def _raw_gn3s(prn, code_phase_chips, doppler, n_blocks, seed):
    """Real 4 Msps samples of a C/A signal at 2.42 MHz + doppler, quantised to the
    GN3S 2-bit codes (0..3 <-> -3, -1, 1, 3)."""
    rng = np.random.default_rng(seed)
    fs, n = 4.0e6, n_blocks * 20000
    t = np.arange(n) / fs
    chips = S.ca_chips(prn).astype(np.float64) * 2 - 1
    idx = np.floor((t * 1.023e6 * (1 + doppler / 1.57542e9) + code_phase_chips)) % 1023
    x = 0.5 * chips[idx.astype(int)] * np.cos(2 * np.pi * (2.42e6 + doppler) * t) \
        + rng.normal(0, 1.0, n)
    return np.digitize(x, [-1.0, 0.0, 1.0]).astype(np.uint8)


def test_raw_bytes_to_acquisition(gpu, oracle):
    """2-bit bytes -> GN3S front end -> strong acquisition, all on the device,
    equal to the oracle chain, and the planted PRN found."""
    o = S.OracleSDR()
    codes = gpu.sdr_prn_codes()
    raw = _raw_gn3s(prn=7, code_phase_chips=300.0, doppler=2000.0, n_blocks=1, seed=5)
    fe = gpu.SdrFeCtx()
    d_in = gpu.DevBuf.from_array(gpu.pack_2bit(raw))
    d_out = gpu.DevBuf(10240 * 4)
    fe.gn3s_dev(d_in.ptr, True, 1, 0, d_out.ptr)
    fe.sync()
    acq = gpu.SdrAcqCtx(38400.0)
    svs = np.arange(32, dtype=np.int32)
    d_svs = gpu.DevBuf.from_array(svs)
    d_res = gpu.DevBuf(5 * 32 * gpu.SDR_RESULT.itemsize)
    acq.strong_dev(d_out.ptr, 5, 32, d_svs.ptr, d_res.ptr)   # the 5 packets of the block
    acq.sync()
    got = d_res.download(np.uint8).view(gpu.SDR_RESULT).reshape(5, 32)
    pk, _ = o.gn3s(raw, 0)
    for r in range(5):
        want = o.acq_strong(pk[r * 2048:(r + 1) * 2048], codes, svs)
        for f in ("sv", "code_phase", "doppler", "magnitude", "row"):
            assert (got[r][f] == want[f]).all(), (r, f)
    best = got[0][np.argmax(got[0]["magnitude"])]
    assert int(best["sv"]) == 6 and abs(int(best["doppler"]) - 2000) <= 250
