"""GPU parity: 2-bit packed IF input (GNSSCORR_IF_PACKED2, the GN3S LUT
{-3,-1,1,3} of GPS_SDR_REAL_TIME_GPS_RECEIVER/objects/gps_source.cpp:692).

A packed stream is the int8 stream of the same levels in a quarter of the
bytes, so every result must be IDENTICAL to the int8 path on the unpacked
samples (which the other GPU tests pin to the reference): tracking results,
dumps and channel state bit-exact; acquisition rows and decisions bit-exact
(same fp64 / fp32 arithmetic on the same values).  Covered paths of
osg_track_kernel: staged shared streams (the channels of one receiver),
unstaged one-stream-per-channel runs (C_s = 1), tail runs (nsamp not a multiple
of 64, odd nsamp), the per-sample path (slews beyond the LDS-staged E/P/L row)
and I-only streams; plus a few channels against the scalar oracle directly.
"""
import numpy as np
import pytest

import osg_scenarios as S
from test_track_gpu import _oracle_channels, _random_cmds

pytestmark = pytest.mark.gpu


def _layout(streams, stride_elems):
    buf = np.zeros(stride_elems * len(streams), np.int8)
    buf[:] = 1                      # a valid level in the padding (packable)
    for i, s in enumerate(streams):
        buf[i * stride_elems: i * stride_elems + len(s)] = s
    return buf


def _pair(gpu, C, nsamp, iq, **kw):
    a = gpu.TrackCtx(C, iq=iq, max_nsamp=nsamp, **kw)
    b = gpu.TrackCtx(C, iq=iq, max_nsamp=nsamp, packed=True, **kw)
    return a, b


def _same(ra, rb):
    for k in ("n_dumps", "dump", "msbit_reg", "tic", "tic_regs"):
        np.testing.assert_array_equal(ra[k], rb[k], err_msg=k)


def _same_state(a, b):
    sa, sb = a.get_state(), b.get_state()
    for k in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc", "ms_counter",
              "bit_counter", "msbit_reg"):
        np.testing.assert_array_equal(sa[k], sb[k], err_msg=k)


@pytest.mark.parametrize("layout", ["receivers", "own_stream"])
@pytest.mark.parametrize("nsamp", [16368, 8184, 8191])
def test_track_packed_equals_int8(gpu, layout, nsamp):
    """Host API, several calls, all dumps: packed == int8 bit-exact."""
    rng = np.random.default_rng(nsamp + len(layout))
    n_calls = 3
    if layout == "receivers":          # 12 channels per stream: staged, shared in LDS
        C, n_streams = 96, 8
        stream_of = np.arange(C) // 12
    else:                              # C_s = 1: unstaged packed runs
        C, n_streams = 64, 64
        stream_of = np.arange(C)
    streams = [S.synth_if(nsamp * n_calls, 300 + i, [(i % 32 + 1, 37 * i, 0, 3)])
               for i in range(n_streams)]
    stride = ((nsamp * n_calls * 2 + 63) // 64) * 64 // 2           # samples
    buf = _layout(streams, stride * 2)
    cmds = _random_cmds(rng, n_calls, C, n_streams, slew=True)
    for k in range(n_calls):
        cmds[k]["stream"] = stream_of
    a, b = _pair(gpu, C, nsamp, True)
    for k in range(n_calls):
        off = k * nsamp * 2                                  # elements
        chunk8 = buf[off:]
        chunkp = gpu.pack2(chunk8)
        ra, _, da = a.track(chunk8, nsamp, cmds[k], n_streams=n_streams, stream_stride=stride,
                            all_dumps=True)
        rb, _, db = b.track(chunkp, nsamp, cmds[k], n_streams=n_streams, stream_stride=stride,
                            all_dumps=True)
        _same(ra, rb)
        for c in range(C):     # entries beyond n_dumps are not written (undefined)
            nd = ra["n_dumps"][c]
            np.testing.assert_array_equal(da[c, :nd], db[c, :nd], err_msg=f"dumps ch{c}")
    _same_state(a, b)


def test_track_packed_vs_oracle(gpu, oracle):
    """A packed run checked against the scalar oracle itself (not only via int8)."""
    rng = np.random.default_rng(11)
    C, n_streams, n_calls, nsamp = 24, 2, 3, 8380
    streams = [S.synth_if(nsamp * n_calls, 500 + i, [(i + 3, 21 * i, 0, 3)])
               for i in range(n_streams)]
    cmds = _random_cmds(rng, n_calls, C, n_streams, slew=True)
    ref, ref_nd, ref_state = _oracle_channels(oracle, streams, nsamp, cmds)
    stride = ((nsamp * n_calls * 2 + 63) // 64) * 64 // 2
    buf = _layout(streams, stride * 2)
    ctx = gpu.TrackCtx(C, iq=True, max_nsamp=nsamp, packed=True)
    for k in range(n_calls):
        res, _ = ctx.track(gpu.pack2(buf[k * nsamp * 2:]), nsamp, cmds[k], n_streams=n_streams,
                           stream_stride=stride)
        nd = (res["n_dumps"] > 0).astype(np.int32)
        np.testing.assert_array_equal(nd, ref_nd[k])
        np.testing.assert_array_equal(res["dump"][nd == 1], ref[k][nd == 1])
    st = ctx.get_state()
    for c in range(C):
        for key in ("carrier_phase", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][c], ref_state[c][key][0], err_msg=f"{key} {c}")


def test_track_packed_big_slew_and_real(gpu):
    """Per-sample paths: slews beyond the LDS-staged row (IQ) and I-only streams."""
    rng = np.random.default_rng(5)
    C, nsamp, n_calls = 48, 16368, 3
    for iq in (True, False):
        IF = S.synth_if(nsamp * n_calls, 9, [(7, 100, 0, 3)], iq=iq)
        cmds = _random_cmds(rng, n_calls, C, 1)
        cmds["slew"][:, ::3] = 1500 + rng.integers(0, 60000, size=(n_calls, C // 3 + (C % 3 > 0)))
        a, b = _pair(gpu, C, nsamp, iq)
        bps = 2 if iq else 1
        for k in range(n_calls):
            seg = IF[k * nsamp * bps:(k + 1) * nsamp * bps]
            ra, _ = a.track(seg, nsamp, cmds[k])
            rb, _ = b.track(gpu.pack2(seg), nsamp, cmds[k])
            _same(ra, rb)
        _same_state(a, b)


def test_track_packed_device_replay(gpu):
    """Device-resident packed IF through replay_dev (k-th call at k*nsamp/2 bytes:
    8184 bytes per 1-ms call at 16.368 Msps, so odd calls start 8-byte aligned)."""
    rng = np.random.default_rng(21)
    C, K, nsamp = 256, 4, 16368
    IF = S.synth_if(nsamp * K, 31, [(2, 7, 0, 3)])
    cmds = _random_cmds(rng, K, C, 1)
    a, b = _pair(gpu, C, nsamp, True)
    assert b.if_bytes(nsamp) == nsamp // 2 and a.if_bytes(nsamp) == 2 * nsamp
    d8, dp = gpu.DevBuf.from_array(IF), gpu.DevBuf.from_array(gpu.pack2(IF))
    dc = gpu.DevBuf.from_array(cmds)
    r8, rp = (gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize) for _ in range(2))
    a.replay_dev(d8.ptr, 0, nsamp, K, dc.ptr, r8.ptr)
    b.replay_dev(dp.ptr, 0, nsamp, K, dc.ptr, rp.ptr)
    a.sync()
    b.sync()
    np.testing.assert_array_equal(r8.download(gpu.TRACK_RESULT), rp.download(gpu.TRACK_RESULT))
    _same_state(a, b)


def test_track_packed_alignment_refused(gpu):
    ctx = gpu.TrackCtx(4, iq=True, max_nsamp=1024, packed=True)
    d = gpu.DevBuf(1 << 16)
    cm = _random_cmds(np.random.default_rng(0), 1, 4, 2)[0]
    dc, dr = gpu.DevBuf.from_array(cm), gpu.DevBuf(4 * gpu.TRACK_RESULT.itemsize)
    with pytest.raises(gpu.GnssCorrError):   # 8 samples = 4 packed bytes: not 8-byte aligned
        ctx.track_dev(d.ptr, 8, 1024, dc.ptr, dr.ptr)


# ---------------------------------------------------------------- acquisition
@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("iq", [True, False])
def test_acq_packed_equals_int8(gpu, prec, iq):
    """acquisition.sci search on packed IF == the int8 search, bit for bit."""
    import acq_oracle
    fs, n = 16.368e6, 16368
    sigs = [dict(system=0, prn=p, code_phase=123.5 + 900 * p, doppler=-1500.0 + 500 * p,
                 cn0=48.0) for p in (3, 11)]
    IF = gpu.ifgen(2 * n, sigs, fs=fs, iq=iq)
    codes = np.stack([acq_oracle.make_ca_table_row(p, fs) for p in (3, 7, 11)])
    freqs = 2.42e6 + np.arange(-5, 6) * 500.0
    gcode = np.arange(3, dtype=np.int32)
    gfreq = np.tile(np.arange(len(freqs), dtype=np.int32), (3, 1))
    out = []
    for packed in (False, True):
        ctx = gpu.AcqCtx(fs, n, precision=prec, max_freqs=16, max_blocks=4, max_codes=4)
        ctx.set_codes(codes)
        src = gpu.pack2(IF) if packed else IF
        out.append(ctx.search(src, 2, freqs, gcode, gfreq, iq=gpu.iq_flags(iq, packed)))
    (r0, w0), (r1, w1) = out
    assert r0.tobytes() == r1.tobytes()
    assert w0.tobytes() == w1.tobytes()
    assert r0["code_phase"][0] > 0


def test_acq_packed_coherent_5ms(gpu):
    """GLONASS-style 5-ms coherent blocks read from packed bytes."""
    import acq_oracle
    fs, n = 16.368e6, 16368
    IF = gpu.ifgen(10 * n, [dict(system=0, prn=5, code_phase=4000.0, doppler=700.0, cn0=44.0)],
                   fs=fs)
    codes = acq_oracle.make_ca_table_row(5, fs)[None]
    freqs = 2.42e6 + np.arange(-4, 5) * 100.0
    res = []
    for packed in (False, True):
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=10, max_codes=2)
        ctx.set_codes(codes)
        ctx.set_coherent(5)
        src = gpu.pack2(IF) if packed else IF
        res.append(ctx.search(src, 2, freqs, np.zeros(1, np.int32),
                              np.arange(len(freqs), dtype=np.int32)[None],
                              iq=gpu.iq_flags(True, packed)))
    assert res[0][0].tobytes() == res[1][0].tobytes()
    assert res[0][1].tobytes() == res[1][1].tobytes()


def test_acq_bad_format_flags(gpu):
    ctx = gpu.AcqCtx(16.368e6, 16368, max_freqs=4, max_blocks=2, max_codes=1)
    import acq_oracle
    ctx.set_codes(acq_oracle.make_ca_table_row(1, 16.368e6)[None])
    with pytest.raises(gpu.GnssCorrError):
        ctx.search(np.zeros(2 * 16368 * 2, np.int8), 1, [2.42e6], [0], [[0]], iq=5)
