"""GPU parity: HIP tracking correlator vs the reference semantics.

* OSG register-level shim (Sim_GP2021_int on the GPU) replays every golden
  scenario bit-exact: all 256 REG_read words after every call and the final
  gp2021_channel state (reference correlator.c:148-316 via
  tests/golden/make_osg_golden.py).
* Batched API with hundreds of channels on several IF streams vs the scalar
  oracle (oracle/osg_corr.c, itself pinned to the reference).
* Size-independent properties at full size: chunking invariance (one 1-ms
  call == two 0.5-ms calls), replay == sequential calls, zero IF -> zero sums.
"""
import os

import numpy as np
import pytest

import osg_scenarios as S

GOLD = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(S.SCENARIOS))
def test_osg_shim_matches_golden(gpu, name):
    scn = S.get(name)
    g = np.load(os.path.join(GOLD, f"osg_{name}.npz"))
    osg = gpu.OSG(samp_rate=16.0e6, n_channels=12, use_iq=scn["iq"])
    for k in range(256):
        osg.REG_read[k] = 0
        osg.REG_write[k] = 0
    osg.correlator_init(scn["tic_period"])
    regs, st = S.run(osg, scn)
    bad = np.argwhere(regs != g["reg_read"])
    assert bad.size == 0, f"first mismatches (call, reg): {bad[:8].tolist()}"
    for k in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
        np.testing.assert_array_equal(st[k], g[k], err_msg=k)


def _oracle_channels(oracle, if_streams, nsamp, cmds_per_call, iq=True):
    """Run each batched channel through its own emulated GP2021 (channel 0)."""
    n_calls, C = cmds_per_call.shape
    out = np.zeros((n_calls, C, 6), np.int32)
    nd = np.zeros((n_calls, C), np.int32)
    state = []
    bps = 2 if iq else 1
    for c in range(C):
        o = oracle.OracleOSG(1, iq, 16.368e6, 0.0)
        rw = o.REG_write
        rw[7] = -1
        for k in range(n_calls):
            cm = cmds_per_call[k, c]
            rw[0] = cm["prn"]
            rw[3], rw[4] = int(cm["carrier_incr"]) >> 16, int(cm["carrier_incr"]) & 0xFFFF
            rw[5], rw[6] = int(cm["code_incr"]) >> 16, int(cm["code_incr"]) & 0xFFFF
            rw[0x84] = cm["slew"]
            s = if_streams[cm["stream"]]
            o.sim(s[k * nsamp * bps:(k + 1) * nsamp * bps], nsamp)
            if o.REG_read[0x82] & 1:
                nd[k, c] = 1
                out[k, c] = o.REG_read[0x84:0x8A]
        state.append(o.chan_state())
    return out, nd, state


def _random_cmds(rng, n_calls, C, n_streams, slew=False):
    cmds = np.zeros((n_calls, C), np.dtype(
        [("prn", "<i4"), ("carrier_incr", "<u4"), ("code_incr", "<u4"), ("slew", "<u4"),
         ("epoch_load", "<i4"), ("stream", "<i4")]))
    prn = rng.integers(0, 33, size=C)
    stream = rng.integers(0, n_streams, size=C)
    for k in range(n_calls):
        cmds[k]["prn"] = prn
        cmds[k]["stream"] = stream
        cmds[k]["carrier_incr"] = 635008600 + rng.integers(-2_000_000, 2_000_000, size=C)
        cmds[k]["code_incr"] = (6710886 + rng.integers(-100, 100, size=C)) * 40
        cmds[k]["slew"] = rng.integers(0, 30, size=C) * (rng.random(C) < 0.2) if slew else 0
        cmds[k]["epoch_load"] = -1
    return cmds


@pytest.mark.parametrize("nsamp", [16368, 8380, 5000, 8381, 2043])
def test_batched_many_channels_vs_oracle(gpu, oracle, nsamp):
    rng = np.random.default_rng(7 + nsamp)
    C, n_streams, n_calls = 96, 3, 4
    streams = [S.synth_if(nsamp * n_calls, 100 + i, [(i + 1, 50 * i, 0, 3)]) for i in range(n_streams)]
    cmds = _random_cmds(rng, n_calls, C, n_streams, slew=True)
    ref, ref_nd, ref_state = _oracle_channels(oracle, streams, nsamp, cmds)
    ctx = gpu.TrackCtx(C, iq=True, max_nsamp=nsamp)
    # streams laid out with a 16-byte aligned stride
    stride = ((nsamp * n_calls * 2 + 15) // 16) * 16 // 2
    buf = np.zeros(stride * 2 * n_streams, np.int8)
    for i, s in enumerate(streams):
        buf[i * stride * 2: i * stride * 2 + len(s)] = s
    for k in range(n_calls):
        # each call reads its chunk: advance the base by k*nsamp samples
        chunk = buf[k * nsamp * 2:]
        res, _ = ctx.track(chunk, nsamp, cmds[k], n_streams=n_streams, stream_stride=stride)
        got_nd = (res["n_dumps"] > 0).astype(np.int32)
        np.testing.assert_array_equal(got_nd, ref_nd[k])
        m = got_nd == 1
        np.testing.assert_array_equal(res["dump"][m], ref[k][m])
    st = ctx.get_state()
    for c in range(C):
        for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][c], ref_state[c][key][0], err_msg=f"{key} ch{c}")


@pytest.mark.parametrize("per_channel_layout", [False, True])
def test_one_stream_per_channel_vs_oracle(gpu, oracle, per_channel_layout):
    """C_s = 1 (every channel its own int8 stream), with and without the
    gnsscorr_track_set_layout hint (per-channel LDS staging): bit-exact either way."""
    rng = np.random.default_rng(31)
    C, nsamp, n_calls = 48, 16368, 2
    streams = [S.synth_if(nsamp * n_calls, 300 + i, [(i % 32 + 1, 37 * i, 0, 3)]) for i in range(C)]
    cmds = _random_cmds(rng, n_calls, C, C)
    for k in range(n_calls):
        cmds[k]["stream"] = np.arange(C)
    ref, ref_nd, ref_state = _oracle_channels(oracle, streams, nsamp, cmds)
    ctx = gpu.TrackCtx(C, iq=True, max_nsamp=nsamp)
    ctx.set_layout(per_channel_layout)
    stride = ((nsamp * n_calls * 2 + 15) // 16) * 16 // 2
    buf = np.zeros(stride * 2 * C, np.int8)
    for i, st in enumerate(streams):
        buf[i * stride * 2: i * stride * 2 + len(st)] = st
    for k in range(n_calls):
        res, _ = ctx.track(buf[k * nsamp * 2:], nsamp, cmds[k], n_streams=C, stream_stride=stride)
        got_nd = (res["n_dumps"] > 0).astype(np.int32)
        np.testing.assert_array_equal(got_nd, ref_nd[k])
        m = got_nd == 1
        np.testing.assert_array_equal(res["dump"][m], ref[k][m])
    st = ctx.get_state()
    for c in range(C):
        for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][c], ref_state[c][key][0], err_msg=f"{key} ch{c}")


# code NCO words for low sample rates: at fs = 4.092 Msps a half-chip is 2
# samples (kinc2 = 2^31), at 2.048 Msps about one (kinc2 ~ 0.999 * 2^32).  There
# an epoch of D >= 2046 half-chips can be as short as a piece-path lane's span
# of 2080 samples (two 32-sample pieces 2048 apart), so those channels must
# not take the per-wave piece path (track.hip: s_short).
LOW_RATES = {"4.092": 1 << 30, "2.048": int(round((1 << 31) * 2.046 / 2.048))}


def _low_rate_cmds(rng, n_calls, C, code_incr, slews):
    cmds = _random_cmds(rng, n_calls, C, C)
    for k in range(n_calls):
        cmds[k]["stream"] = np.arange(C)
        cmds[k]["code_incr"] = code_incr + rng.integers(-20000, 20000, size=C)
        cmds[k]["slew"] = slews
    return cmds


def _layout_streams(streams, nsamp, n_calls):
    stride = ((nsamp * n_calls * 2 + 63) // 64) * 64 // 2
    buf = np.ones(stride * 2 * len(streams), np.int8)
    for i, st in enumerate(streams):
        buf[i * stride * 2: i * stride * 2 + len(st)] = st
    return buf, stride


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("rate", sorted(LOW_RATES))
@pytest.mark.parametrize("nsamp", [5000, 16368])
def test_low_rate_one_stream_per_channel_all_dumps_vs_oracle(gpu, oracle, rate, nsamp, packed):
    """C_s = 1 at 4.092 / 2.048 Msps code rates, no slew: EVERY dump of every
    call equals the oracle's (its dump log: REG_read latches only the last)."""
    rng = np.random.default_rng(11 + nsamp + 3 * packed)
    C, n_calls = 40, 2
    streams = [S.synth_if(nsamp * n_calls, 500 + i, [(i % 32 + 1, 37 * i, 0, 3)]) for i in range(C)]
    cmds = _low_rate_cmds(rng, n_calls, C, LOW_RATES[rate], 0)
    buf, stride = _layout_streams(streams, nsamp, n_calls)
    ctx = gpu.TrackCtx(C, iq=True, max_nsamp=nsamp, packed=packed)
    got = []
    for k in range(n_calls):
        chunk = buf[k * nsamp * 2:]
        res, _, d = ctx.track(gpu.pack2(chunk) if packed else chunk, nsamp, cmds[k], n_streams=C,
                              stream_stride=stride, all_dumps=True)
        got.append((res["n_dumps"].copy(), d.copy()))
    st = ctx.get_state()
    multi = 0
    for c in range(C):
        o = oracle.OracleOSG(1, True, 16.368e6, 0.0)
        rw = o.REG_write
        rw[7] = -1
        for k in range(n_calls):
            cm = cmds[k, c]
            rw[0] = cm["prn"]
            rw[3], rw[4] = int(cm["carrier_incr"]) >> 16, int(cm["carrier_incr"]) & 0xFFFF
            rw[5], rw[6] = int(cm["code_incr"]) >> 16, int(cm["code_incr"]) & 0xFFFF
            rw[0x84] = 0
            want = o.sim_dumps(streams[c][k * nsamp * 2:(k + 1) * nsamp * 2], nsamp)[:, 1:]
            nd, d = got[k]
            assert nd[c] == len(want), (c, k, nd[c], len(want))
            np.testing.assert_array_equal(d[c, :nd[c]], want, err_msg=f"ch{c} call{k}")
            multi += len(want) >= 2
        ref = o.chan_state()
        for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][c], ref[key][0], err_msg=f"{key} ch{c}")
    if not (rate == "4.092" and nsamp < 8184):   # (a 4092-sample epoch: 1-2 per call)
        assert multi >= C // 2      # most calls of active channels hold several dumps


@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("rate", sorted(LOW_RATES))
def test_low_rate_one_stream_per_channel_slews_vs_oracle(gpu, oracle, rate, packed):
    """Same rates with slews around the piece path's limit (D = 2046 + slew
    against a 2080-sample lane span) and beyond the staged E/P/L row: last dump,
    dump flags and channel state bit-exact over 3 calls of 16368 samples."""
    rng = np.random.default_rng(23 + 5 * packed)
    C, nsamp, n_calls = 42, 16368, 3
    streams = [S.synth_if(nsamp * n_calls, 700 + i, [(i % 32 + 1, 41 * i, 0, 3)]) for i in range(C)]
    slews = np.resize(np.array([0, 30, 34, 35, 36, 40, 200, 1100, 3000], np.uint32), C)
    cmds = _low_rate_cmds(rng, n_calls, C, LOW_RATES[rate], slews)
    ref, ref_nd, ref_state = _oracle_channels(oracle, streams, nsamp, cmds)
    buf, stride = _layout_streams(streams, nsamp, n_calls)
    ctx = gpu.TrackCtx(C, iq=True, max_nsamp=nsamp, packed=packed)
    for k in range(n_calls):
        chunk = buf[k * nsamp * 2:]
        res, _ = ctx.track(gpu.pack2(chunk) if packed else chunk, nsamp, cmds[k], n_streams=C,
                           stream_stride=stride)
        got_nd = (res["n_dumps"] > 0).astype(np.int32)
        np.testing.assert_array_equal(got_nd, ref_nd[k])
        m = got_nd == 1
        np.testing.assert_array_equal(res["dump"][m], ref[k][m])
    st = ctx.get_state()
    for c in range(C):
        for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][c], ref_state[c][key][0], err_msg=f"{key} ch{c}")


def test_chunking_invariance_full_size(gpu):
    """One 16368-sample call == two 8184-sample calls (4096 channels)."""
    rng = np.random.default_rng(3)
    C = 4096
    IF = S.synth_if(16368, 5, [(3, 100, 0, 3)])
    cm = _random_cmds(rng, 1, C, 1)[0]
    a = gpu.TrackCtx(C, max_nsamp=16368)
    b = gpu.TrackCtx(C, max_nsamp=16368)
    ra, _, da = a.track(IF, 16368, cm, all_dumps=True)
    rb1, _, db1 = b.track(IF[:16368], 8184, cm, all_dumps=True)
    rb2, _, db2 = b.track(IF[16368:], 8184, cm, all_dumps=True)
    sa, sb = a.get_state(), b.get_state()
    for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
        np.testing.assert_array_equal(sa[key], sb[key], err_msg=key)
    # dumps: concatenation of the two halves' dumps equals the single call's
    for c in range(0, C, 97):
        da_c = da[c, :ra["n_dumps"][c]]
        db_c = np.concatenate([db1[c, :rb1["n_dumps"][c]], db2[c, :rb2["n_dumps"][c]]])
        np.testing.assert_array_equal(da_c, db_c)


def test_zero_if_gives_zero(gpu):
    C = 64
    ctx = gpu.TrackCtx(C, max_nsamp=16368)
    cm = _random_cmds(np.random.default_rng(1), 1, C, 1)[0]
    for _ in range(3):
        res, _ = ctx.track(np.zeros(16368 * 2, np.int8), 16368, cm)
    assert (res["dump"] == 0).all()
    assert (ctx.get_state()["acc"] == 0).all()


def test_replay_equals_sequential(gpu):
    rng = np.random.default_rng(9)
    C, K, nsamp = 256, 6, 16368
    IF = S.synth_if(nsamp * K, 77, [(5, 10, 0, 3)])
    cmds = _random_cmds(rng, K, C, 1)
    seq = gpu.TrackCtx(C, max_nsamp=nsamp)
    seq_res = []
    for k in range(K):
        r, _ = seq.track(IF[k * nsamp * 2:(k + 1) * nsamp * 2], nsamp, cmds[k])
        seq_res.append(r)
    rep = gpu.TrackCtx(C, max_nsamp=nsamp)
    d_if = gpu.DevBuf.from_array(IF)
    d_cmds = gpu.DevBuf.from_array(cmds)
    d_res = gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize)
    rep.replay_dev(d_if.ptr, 0, nsamp, K, d_cmds.ptr, d_res.ptr)
    rep.sync()
    got = d_res.download(gpu.TRACK_RESULT).reshape(K, C)
    for k in range(K):
        np.testing.assert_array_equal(got[k]["n_dumps"], seq_res[k]["n_dumps"])
        np.testing.assert_array_equal(got[k]["dump"], seq_res[k]["dump"])
    np.testing.assert_array_equal(rep.get_state()["acc"], seq.get_state()["acc"])


def test_replay_prn_and_slew_change_between_calls(gpu):
    """n calls in one osg_stream_kernel launch keep a channel's staged E/P/L row while
    its PRN and the row's reach stay the same: calls that switch PRN (or go idle and
    come back) or raise the slew must restage it -- equal to one call per launch."""
    rng = np.random.default_rng(21)
    C, K, nsamp = 96, 5, 16368
    IF = S.synth_if(nsamp * K, 78, [(3, 20, 0, 3)])
    cmds = _random_cmds(rng, K, C, 1, slew=True)
    for k in range(1, K):
        sw = rng.random(C) < 0.3
        cmds[k]["prn"][sw] = rng.integers(0, 33, sw.sum())
        cmds[k]["slew"] = np.where(rng.random(C) < 0.3, rng.integers(0, 1200, C), cmds[k]["slew"])
    seq = gpu.TrackCtx(C, max_nsamp=nsamp)
    seq_res = []
    for k in range(K):
        r, _ = seq.track(IF[k * nsamp * 2:(k + 1) * nsamp * 2], nsamp, cmds[k])
        seq_res.append(r)
    rep = gpu.TrackCtx(C, max_nsamp=nsamp)
    d_if = gpu.DevBuf.from_array(IF)
    d_cmds = gpu.DevBuf.from_array(cmds)
    d_res = gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize)
    rep.replay_dev(d_if.ptr, 0, nsamp, K, d_cmds.ptr, d_res.ptr)
    rep.sync()
    got = d_res.download(gpu.TRACK_RESULT).reshape(K, C)
    for k in range(K):
        assert got[k].tobytes() == seq_res[k].tobytes(), k
    for f in ("carrier_phase", "code_phase", "half_chip", "acc", "ms_counter"):
        np.testing.assert_array_equal(rep.get_state()[f], seq.get_state()[f])


def _unpack2(b):
    """GNSSCORR_IF_PACKED2 bytes -> int8 levels (element e: bits 2(e%4) of byte e/4)."""
    b = np.asarray(b, np.uint8)
    codes = (b[:, None] >> (2 * np.arange(4, dtype=np.uint8))) & 3
    return (2 * codes.astype(np.int8) - 3).ravel()


@pytest.mark.parametrize("packed", [False, True], ids=["int8", "packed2"])
def test_replay_many_streams_equals_single_calls(gpu, oracle, packed):
    """The bench's C_s = 1 shape: 3072 channels, one IF stream each at a nonzero
    stride, 10 calls in ONE replay_dev launch, with channels that switch stream, go
    idle or change PRN between calls (the cross-call prefetch then reads another
    stream's first piece).  Byte-identical to 10 single-call launches; 64 channels
    spot-checked against the scalar oracle (oracle/osg_corr.c)."""
    rng = np.random.default_rng(31 + packed)
    C, K, nsamp = 3072, 10, 16368
    stride = K * nsamp + 64                         # samples per stream (not a multiple of nsamp)
    rep = gpu.TrackCtx(C, max_nsamp=nsamp, packed=packed)
    seq = gpu.TrackCtx(C, max_nsamp=nsamp, packed=packed)
    sb = rep.if_bytes(stride)
    d_if = gpu.DevBuf(C * sb + 64)
    d_if.fill_if2(0x5EED00A0 + packed)
    cmds = _random_cmds(rng, K, C, C)
    cmds[0]["stream"] = np.arange(C)
    for k in range(1, K):
        cmds[k]["stream"] = cmds[k - 1]["stream"]
        sw = rng.random(C) < 0.1                    # another stream from this call on
        cmds[k]["stream"][sw] = rng.integers(0, C, sw.sum())
        idle = rng.random(C) < 0.05                 # idle for a call
        cmds[k]["prn"][idle] = 0
        np_ = rng.random(C) < 0.05                  # a new PRN
        cmds[k]["prn"][np_] = rng.integers(1, 33, np_.sum())
    d_cmds = gpu.DevBuf.from_array(cmds)
    d_res = gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize)
    rep.replay_dev(d_if.ptr, stride, nsamp, K, d_cmds.ptr, d_res.ptr)
    rep.sync()
    got = d_res.download(gpu.TRACK_RESULT).reshape(K, C)
    d_r1 = gpu.DevBuf(C * gpu.TRACK_RESULT.itemsize)
    for k in range(K):
        # one call per launch: the IF of call k starts k * nsamp samples into every stream
        seq.track_dev(d_if.ptr + seq.if_bytes(k * nsamp), stride, nsamp,
                      d_cmds.ptr + k * C * gpu.NCO_CMD.itemsize, d_r1.ptr, 0, seq.next_tic(nsamp))
        seq.sync()
        r = d_r1.download(gpu.TRACK_RESULT)
        assert got[k].tobytes() == r.tobytes(), \
            (k, np.flatnonzero((got[k]["dump"] != r["dump"]).any(axis=1))[:8])
    sr, ss = rep.get_state(), seq.get_state()
    for f in sr.dtype.names:
        np.testing.assert_array_equal(sr[f], ss[f], err_msg=f)
    # oracle spot check: 64 channels, their streams downloaded (and unpacked)
    sel = np.sort(rng.choice(C, 64, replace=False))
    used = np.unique(cmds[:, sel]["stream"])
    host = {}
    for s in used:
        raw = d_if.download(np.int8 if not packed else np.uint8, sb, int(s) * sb)
        host[int(s)] = _unpack2(raw)[:2 * stride] if packed else raw
    sub = cmds[:, sel].copy()
    want, nd, ref_state = _oracle_channels(oracle, host, nsamp, sub)
    for k in range(K):
        g = got[k][sel]
        np.testing.assert_array_equal((g["n_dumps"] > 0).astype(np.int32), nd[k])
        m = nd[k] == 1
        np.testing.assert_array_equal(g["dump"][m], want[k][m])
    st = rep.get_state()[sel]
    for j in range(len(sel)):
        for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][j], ref_state[j][key][0], err_msg=f"{key} {j}")


def test_replay_bench_receiver_shape(gpu, oracle):
    """The bench's main tracking shape: 1024 receivers x 12 channels
    = 12288 channel-waves on 1024 interleaved int8 IQ streams, the bench's NCO schedule
    (+-5 kHz carrier, +-3 ppm code Doppler, bench.py _track_cmds), 10 calls in ONE
    replay_dev launch.  At this size the XCD mapping and the LDS balance padding depend
    on the workgroup count, so it gets its own check: byte-identical to 10 single-call
    launches, and 64 channels against the scalar oracle (oracle/osg_corr.c, reference
    OSG/correlator/correlator.c:149-316)."""
    rng = np.random.default_rng(12288)
    RX, CH, K, nsamp = 1024, 12, 10, 16368
    C = RX * CH
    stride = K * nsamp
    rep = gpu.TrackCtx(C, max_nsamp=nsamp, samp_rate=16.368e6)
    seq = gpu.TrackCtx(C, max_nsamp=nsamp, samp_rate=16.368e6)
    sb = rep.if_bytes(stride)
    d_if = gpu.DevBuf(RX * sb)
    d_if.fill_if2(0x5EED0003)
    cmd1 = np.zeros(C, gpu.NCO_CMD)
    cmd1["prn"] = rng.integers(1, 33, C)
    cmd1["stream"] = np.repeat(np.arange(RX), CH)
    cmd1["carrier_incr"] = 635008600 + rng.integers(-262000, 262000, C) * 20
    cmd1["code_incr"] = 6710886 * 40 + rng.integers(-800, 800, C)
    cmd1["epoch_load"] = -1
    cmds = np.tile(cmd1, K).reshape(K, C)
    d_cmds = gpu.DevBuf.from_array(cmds)
    d_res = gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize)
    rep.replay_dev(d_if.ptr, stride, nsamp, K, d_cmds.ptr, d_res.ptr)
    rep.sync()
    got = d_res.download(gpu.TRACK_RESULT).reshape(K, C)
    d_r1 = gpu.DevBuf(C * gpu.TRACK_RESULT.itemsize)
    for k in range(K):
        seq.track_dev(d_if.ptr + seq.if_bytes(k * nsamp), stride, nsamp,
                      d_cmds.ptr + k * C * gpu.NCO_CMD.itemsize, d_r1.ptr, 0, seq.next_tic(nsamp))
        seq.sync()
        r = d_r1.download(gpu.TRACK_RESULT)
        assert got[k].tobytes() == r.tobytes(), \
            (k, np.flatnonzero((got[k]["dump"] != r["dump"]).any(axis=1))[:8])
    sr, ss = rep.get_state(), seq.get_state()
    for f in sr.dtype.names:
        np.testing.assert_array_equal(sr[f], ss[f], err_msg=f)
    assert (got["n_dumps"] >= 1).sum() >= C * K // 2   # 1-ms calls: most calls dump
    sel = np.sort(rng.choice(C, 64, replace=False))
    host = {int(s): d_if.download(np.int8, sb, int(s) * sb)
            for s in np.unique(cmds[:, sel]["stream"])}
    want, nd, ref_state = _oracle_channels(oracle, host, nsamp, cmds[:, sel].copy())
    for k in range(K):
        g = got[k][sel]
        np.testing.assert_array_equal((g["n_dumps"] > 0).astype(np.int32), nd[k])
        m = nd[k] == 1
        np.testing.assert_array_equal(g["dump"][m], want[k][m])
    st = rep.get_state()[sel]
    for j in range(len(sel)):
        for key in ("carrier_phase", "carrier_cycle", "code_phase", "half_chip", "acc"):
            np.testing.assert_array_equal(st[key][j], ref_state[j][key][0], err_msg=f"{key} {j}")


def test_track_rejects_bad_prn(gpu):
    ctx = gpu.TrackCtx(4, max_nsamp=1024)
    cm = _random_cmds(np.random.default_rng(0), 1, 4, 1)[0]
    cm["prn"][2] = 40
    with pytest.raises(gpu.GnssCorrError):
        ctx.track(np.zeros(2048, np.int8), 1024, cm)


def test_device_lds_bytes(gpu):
    """The LDS a workgroup may allocate, as the per-channel staging fit check reads it
    (gnsscorr_device_lds_bytes): 160 KiB on gfx950."""
    assert gpu.device_lds_bytes(0) >= 160 * 1024
