"""GPU parity: GPS-SDR device-resident closed loop (gnsscorr_sdr_track_dev).

Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/objects/
correlator.cpp (Correlate :160-237, UpdateState :369-422, DumpAccum :452-525,
ProcessFeedback :530-555) driving channel.cpp (Accum :182-279) at every dump.

The device loop must equal the host-scheduled composition of the two pieces
already pinned against the reference (test_sdr_corr_gpu.py: correlator vs
oracle/sdr_corr.c; test_sdr_channel*.py: channel vs the compiled reference):
  * correlator side: gnsscorr_sdr_correlate, packet by packet, with a dump
    callback that replays the device loop's logged feedback -- the rotated
    correlations handed to the callback must equal the logged ones at every
    dump, and final states / correlations must be identical;
  * channel side: the logged correlations fed to gnsscorr_sdr_channel_accum_dev
    in order must give the logged feedback at every call and the same final
    Channel object.
Together: device loop == host Correlate + Channel::Accum callback, bit for bit.
Also: one 400-packet launch == two 200-packet launches; bad receiver index and
out-of-table states stop the channel with a status.
"""
import ctypes as C

import numpy as np
import pytest

from test_sdr_corr_gpu import _scene

pytestmark = pytest.mark.gpu

DUMP_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p)


def _init(gpu, ctx, chans):
    n = len(chans)
    st = np.zeros(n, gpu.SDR_CHAN)
    ch = np.zeros(n, gpu.SDR_CHANNEL)
    for c, (rx, sv, cp, dop) in enumerate(chans):
        st[c] = ctx.init_chan(sv, cp, dop, 3.0)
        ch[c] = ctx.channel_start(c, sv, dop, 1)
    return st, np.zeros(n, gpu.SDR_CORR), ch


def _as(gpu, ptr, dt):
    return np.frombuffer((C.c_char * dt.itemsize).from_address(ptr), dt)[0]


@pytest.fixture(scope="module")
def loop(gpu):
    K = 400
    pk, chans = _scene(K, n_rx=2)
    ctx = gpu.SdrCorrCtx()
    st0, c0, ch0 = _init(gpu, ctx, chans)
    st, corr, ch = st0.copy(), c0.copy(), ch0.copy()
    rx = np.array([c[0] for c in chans], np.int32)
    out = ctx.track(pk, st, corr, ch, rx=rx, log_per_ch=2 * K + 2)
    return dict(K=K, pk=pk, chans=chans, rx=rx, ctx=ctx, st0=st0, ch0=ch0, st=st, corr=corr,
                ch=ch, out=out)


def test_track_correlator_side(gpu, loop):
    L = loop
    log, n_log = L["out"]["log"], L["out"]["n_log"]
    n = len(L["chans"])
    assert (n_log >= 350).sum() >= n - 2, n_log       # ~1 dump per packet per live channel
    st, corr = L["st0"].copy(), np.zeros(n, gpu.SDR_CORR)
    pos = np.zeros(n, np.int64)
    bad = []

    def cb(user, c, s, cr, f):
        i = pos[c]
        pos[c] += 1
        rec = log[c, i]
        got = _as(gpu, cr, gpu.SDR_CORR)
        if got.tobytes() != rec["corr"].tobytes():
            bad.append((c, int(i), got, rec["corr"]))
        C.memmove(f, rec["fb"].tobytes(), gpu.SDR_FEEDBACK.itemsize)

    fn = DUMP_FN(cb)
    for k in range(L["K"]):
        L["ctx"].correlate(L["pk"][k], st, corr, C.cast(fn, C.c_void_p).value, rx=L["rx"])
        assert not bad, (k, bad[:3])
    assert (pos == n_log).all()
    assert st.tobytes() == L["st"].tobytes()
    assert corr.tobytes() == L["corr"].tobytes()
    # the packet / phase bookkeeping of the log is consistent
    for c in range(n):
        p = log[c, :n_log[c]]["packet"]
        assert (np.diff(p) >= 0).all() and (np.bincount(p) <= 2).all()


def test_track_channel_side(gpu, loop):
    L = loop
    log, n_log = L["out"]["log"], L["out"]["n_log"]
    ev_dev = L["out"]["events"]
    ev_host = []
    for c in range(len(L["chans"])):
        m = int(n_log[c])
        if m == 0:
            assert L["ch"][c].tobytes() == L["ch0"][c].tobytes()
            continue
        chc = L["ch0"][c:c + 1].copy()
        cr = log[c, :m]["corr"]
        rows = np.stack([cr["i"][:, 0], cr["i"][:, 1], cr["i"][:, 2],
                         cr["q"][:, 0], cr["q"][:, 1], cr["q"][:, 2]], 1).astype(np.int32)
        fb, ev, _ = L["ctx"].channel_accum(rows.reshape(m, 1, 6), chc)
        assert fb[:, 0].tobytes() == log[c, :m]["fb"].tobytes(), c
        diff = [(f, np.flatnonzero(np.atleast_1d(chc[0][f] != L["ch"][c][f]))[:8])
                for f in gpu.SDR_CHANNEL.names if chc[0][f].tobytes() != L["ch"][c][f].tobytes()]
        assert not diff, (c, diff, chc[0]["fft_buff"][-4:], L["ch"][c]["fft_buff"][-4:],
                          L["ch0"][c]["fft_buff"][-4:])
        ev_host += [(c, int(e["sv"]), int(e["subframe"]), e["word_buff"].tobytes()) for e in ev]
    dev = sorted((int(e["chan"]), int(e["sv"]), int(e["subframe"]), e["word_buff"].tobytes())
                 for e in ev_dev)
    assert dev == sorted(ev_host)


def test_track_split_launches(gpu, loop):
    L = loop
    K = L["K"]
    st, corr, ch = L["st0"].copy(), np.zeros(len(L["chans"]), gpu.SDR_CORR), L["ch0"].copy()
    n1 = L["ctx"].track(L["pk"][:K // 2], st, corr, ch, rx=L["rx"])["events"]
    n2 = L["ctx"].track(L["pk"][K // 2:], st, corr, ch, rx=L["rx"])["events"]
    assert st.tobytes() == L["st"].tobytes()
    assert corr.tobytes() == L["corr"].tobytes()
    assert ch.tobytes() == L["ch"].tobytes()
    assert len(n1) + len(n2) == len(L["out"]["events"])


@pytest.mark.parametrize("cpw", ["5", "7", "16"])
def test_track_channels_per_wave_equal_one(gpu, loop, cpw, monkeypatch):
    """cpw > 1 (several channels per wavefront: each lane runs its channel's
    scalar chain, the wave runs the posted Accum segments one channel after
    the other -- the bench's 3072-channel shape) equals the cpw = 1 launch of
    the fixture bit for bit: states, correlations, Channel objects, the per-dump
    log and the subframe events.  24 channels are not a multiple of 5, 7 or 16,
    so the last wave runs a partial set."""
    L = loop
    monkeypatch.setenv("GNSSCORR_SDR_LOOP_CPW", cpw)
    st, corr, ch = L["st0"].copy(), np.zeros(len(L["chans"]), gpu.SDR_CORR), L["ch0"].copy()
    out = L["ctx"].track(L["pk"], st, corr, ch, rx=L["rx"], log_per_ch=2 * L["K"] + 2)
    assert st.tobytes() == L["st"].tobytes()
    assert corr.tobytes() == L["corr"].tobytes()
    assert ch.tobytes() == L["ch"].tobytes()
    ref = L["out"]
    np.testing.assert_array_equal(out["n_log"], ref["n_log"])
    for c in range(len(L["chans"])):
        m = int(ref["n_log"][c])
        assert out["log"][c, :m].tobytes() == ref["log"][c, :m].tobytes(), c
    key = lambda e: (int(e["chan"]), int(e["sv"]), int(e["subframe"]), e["word_buff"].tobytes())
    assert sorted(map(key, out["events"])) == sorted(map(key, ref["events"]))


def test_track_channel_kill(gpu):
    """A channel killed by the channel (state EMPTY -> kill) stops its correlator
    as ProcessFeedback's memset does; the other channels are unaffected."""
    K = 60
    pk, chans = _scene(K, n_rx=1)
    ctx = gpu.SdrCorrCtx()
    st, corr, ch = _init(gpu, ctx, chans)
    ch[3]["state"] = 0                                 # Error() will kill at the first dump
    st_ref, corr_ref, ch_ref = st.copy(), corr.copy(), ch.copy()
    ctx.track(pk, st, corr, ch)
    assert st[3]["active"] == 0 and st[3]["count"] == 1
    keep = np.arange(len(chans)) != 3
    st2, corr2, ch2 = st_ref[keep].copy(), corr_ref[keep].copy(), ch_ref[keep].copy()
    ctx.track(pk, st2, corr2, ch2)
    assert st2.tobytes() == st[keep].tobytes() and corr2.tobytes() == corr[keep].tobytes()


def test_track_bad_state_stops(gpu):
    ctx = gpu.SdrCorrCtx()
    st = np.zeros(2, gpu.SDR_CHAN)
    st[0] = ctx.init_chan(0, 100, 0)
    st[1] = ctx.init_chan(1, 100, 0)
    st[1]["sbin"] = 5000
    ch = np.zeros(2, gpu.SDR_CHANNEL)
    ch[0] = ctx.channel_start(0, 0, 0, 1)
    ch[1] = ctx.channel_start(1, 1, 0, 1)
    pk = np.zeros((3, 1, 2048, 2), np.int16)
    with pytest.raises(gpu.GnssCorrError, match="channel 1 stopped"):
        ctx.track(pk, st, np.zeros(2, gpu.SDR_CORR), ch)
    with pytest.raises(gpu.GnssCorrError, match="status -1"):
        ctx.track(pk, st[:1].copy(), np.zeros(1, gpu.SDR_CORR), ch[:1].copy(),
                  rx=np.array([1], np.int32))
