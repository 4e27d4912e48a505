"""GPU parity: SoftGNSS float tracking (sgt.hip) vs the fp64 tracking.sci oracle.

Reference: POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/tracking.sci:150-400 and
GPS/L1/tracking.sci:124-360, restated in oracle/sgt_oracle.py (parity unpinned
against a Scilab run).

Tolerances (north_star: integer NCO/code indices bit-exact, float I/Q sums
within 1e-6 relative):
  * blksize, sample position: exact; remCodePhase / remCarrPhase after an
    open-loop epoch: bit-exact (same fp64 operation sequence, no contraction)
  * the six sums: |gpu - ref| <= 1e-6 * |ref| + 1e-6
  * closed loop (the loop filters run on the GPU, fp64 atan/atan2/sqrt may
    differ by an ulp from the host libm): every per-epoch field within
    rel 1e-6 of the oracle over the whole run, blksize exact.
"""
import numpy as np
import pytest

import sgt_oracle as S

pytestmark = pytest.mark.gpu
FS = 16e6
# initSettings.sci's 16 MHz, and BASELINE config 4's 16.368 Msps:
# 32.03 samples per ST chip, so ceil(remCode +- spc + k*step) crosses chip
# boundaries at non-integer sample positions (tracking.sci:281-302)
RATES = [16e6, 16.368e6]
SUMS = ("I_E", "I_P", "I_L", "Q_E", "Q_P", "Q_L")


def _close(a, b, rtol=1e-6, atol=1e-6):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.abs(a - b) <= rtol * np.abs(b) + atol


def _glo_start(cp_chips, fs=FS):
    return int(round((511 - cp_chips) / 0.511e6 * fs)) + 1


@pytest.mark.parametrize("fs", RATES)
@pytest.mark.parametrize("threads", [None, "64", "1024"])
@pytest.mark.parametrize("system,file_type,switch", [(1, 2, 0), (1, 2, 1), (0, 2, 0), (1, 1, 0)])
def test_open_loop_epoch_matches_oracle(gpu, system, file_type, switch, threads, fs, monkeypatch):
    """threads: launch shape override (GNSSCORR_SGT_THREADS; 64 = one wave per channel)."""
    gc = gpu
    if threads:
        monkeypatch.setenv("GNSSCORR_SGT_THREADS", threads)
    rng = np.random.default_rng(17 + system + 3 * file_type + 7 * switch)
    n = 200000
    IF = gc.ifgen(n, [], fs=fs, iq=file_type == 2, seed=21)
    d_if = gc.DevBuf.from_array(IF)
    ctx = gc.SgtCtx(system, fileType=file_type, switchIQ=switch, samplingFreq=fs)
    s = S.settings(system, fileType=file_type, switchIQ=switch, samplingFreq=fs)
    C = 96
    ids = rng.integers(-7, 7, C) if system == 1 else rng.integers(1, 33, C)
    ch = np.zeros(C, gc.SGT_CHAN)
    ch["code_id"] = ids
    ch["pos"] = rng.integers(0, n - 20000, C)
    basis = s["codeFreqBasis"]
    ch["code_freq"] = basis + rng.uniform(-40, 40, C)
    step = ch["code_freq"] / fs
    ch["rem_code"] = rng.uniform(0, 1, C) * step
    ch["rem_carr"] = rng.uniform(-6.2, 6.2, C)
    ch["carr_freq"] = rng.uniform(-3e6, 3e6, C)
    ch0 = ch.copy()
    ep = ctx.track(d_if.ptr, 0, n, ch, 1, closed_loop=False)[:, 0]
    for i in range(C):
        pad = S.padded_code(system, int(ids[i]))
        sums, blk, pos, rc, rcar = S.correlate(IF, s, pad, int(ch0["pos"][i]),
                                               float(ch0["rem_code"][i]),
                                               float(ch0["rem_carr"][i]),
                                               float(ch0["code_freq"][i]),
                                               float(ch0["carr_freq"][i]))
        assert ep["status"][i] == 0 and ep["blksize"][i] == blk
        assert ch["pos"][i] == pos
        assert ch["rem_code"][i] == rc, (i, ch["rem_code"][i], rc)
        assert ch["rem_carr"][i] == rcar, (i, ch["rem_carr"][i], rcar)
        got = np.array([ep[f][i] for f in SUMS])
        assert _close(got, sums).all(), (i, got, sums)
    # frequencies are held in open loop
    assert (ch["carr_freq"] == ch0["carr_freq"]).all()
    assert (ch["code_freq"] == ch0["code_freq"]).all()


@pytest.mark.parametrize("fs", [4.096e6, 2.048e6])
@pytest.mark.parametrize("system", [1, 0])
def test_open_loop_low_rate_unclamped_path(gpu, system, fs):
    """Low sample rates (fewer than ~15 samples per chip): the chunked path does
    not apply and the per-sample index path runs without its clamp (in_table),
    reading the code table by the exact ceil(remCode -/+ spc + k*step) indices;
    remCode over the whole [0, step) range.  Indices and state bit-exact, sums
    within 1e-6 (tracking.sci:281-302)."""
    gc = gpu
    rng = np.random.default_rng(int(fs) % 1000 + system)
    n = int(fs * 0.012)
    IF = gc.ifgen(n, [], fs=fs, seed=44)
    d_if = gc.DevBuf.from_array(IF)
    ctx = gc.SgtCtx(system, samplingFreq=fs)
    s = S.settings(system, samplingFreq=fs)
    C = 64
    ids = rng.integers(-7, 7, C) if system == 1 else rng.integers(1, 33, C)
    ch = np.zeros(C, gc.SGT_CHAN)
    ch["code_id"] = ids
    ch["pos"] = rng.integers(0, n - int(fs * 0.0012), C)
    ch["code_freq"] = s["codeFreqBasis"] + rng.uniform(-40, 40, C)
    step = ch["code_freq"] / fs
    ch["rem_code"] = rng.uniform(0, 1, C) * step
    ch["rem_code"][:4] = 0.0
    ch["rem_code"][4:8] = np.nextafter(step[4:8], 0)
    ch["rem_carr"] = rng.uniform(-6.2, 6.2, C)
    ch["carr_freq"] = rng.uniform(-1e6, 1e6, C)
    ch0 = ch.copy()
    ep = ctx.track(d_if.ptr, 0, n, ch, 1, closed_loop=False)[:, 0]
    for i in range(C):
        pad = S.padded_code(system, int(ids[i]))
        sums, blk, pos, rc, rcar = S.correlate(IF, s, pad, int(ch0["pos"][i]),
                                               float(ch0["rem_code"][i]),
                                               float(ch0["rem_carr"][i]),
                                               float(ch0["code_freq"][i]),
                                               float(ch0["carr_freq"][i]))
        assert ep["status"][i] == 0 and ep["blksize"][i] == blk
        assert ch["pos"][i] == pos and ch["rem_code"][i] == rc and ch["rem_carr"][i] == rcar
        got = np.array([ep[f][i] for f in SUMS])
        assert _close(got, sums).all(), (i, got, sums)


@pytest.mark.parametrize("threads", [None, "64"])
@pytest.mark.parametrize("chunk", ["1", "0"])
@pytest.mark.parametrize("system,file_type", [(1, 2), (0, 2), (1, 1)])
def test_open_loop_crossings_on_exact_chips(gpu, system, file_type, chunk, threads, monkeypatch):
    """codeFreq = fs/32 (GPS: fs/16) and remCode on the 1/32 grid: every code index
    crossing ceil(remCode -/+ spc + k*step) lands exactly on an integer chip.  There
    the chunked paths' real-valued crossing estimates have no margin, so the exact
    reference expression decides (sgt.hip run_chunks; in wave mode, threads "64",
    run_chips' exact chunk boundaries and its per-sample loop for chunks outside the
    capture windows); GNSSCORR_SGT_CHUNK=0 runs the per-sample index path on the same
    inputs.  Indices and state bit-exact."""
    gc = gpu
    monkeypatch.setenv("GNSSCORR_SGT_CHUNK", chunk)
    if threads:
        monkeypatch.setenv("GNSSCORR_SGT_THREADS", threads)
    rng = np.random.default_rng(5 + system + 2 * file_type)
    n = 120000
    IF = gc.ifgen(n, [], fs=FS, iq=file_type == 2, seed=33)
    d_if = gc.DevBuf.from_array(IF)
    ctx = gc.SgtCtx(system, fileType=file_type, samplingFreq=FS)
    s = S.settings(system, fileType=file_type, samplingFreq=FS)
    C = 32
    ids = rng.integers(-7, 7, C) if system == 1 else rng.integers(1, 33, C)
    ch = np.zeros(C, gc.SGT_CHAN)
    ch["code_id"] = ids
    ch["pos"] = rng.integers(0, n - 20000, C)
    ch["code_freq"] = FS / (32 if system == 1 else 16)
    ch["rem_code"] = rng.integers(0, 2, C) / 32.0
    ch["rem_carr"] = rng.uniform(-6.2, 6.2, C)
    ch["carr_freq"] = rng.uniform(-3e6, 3e6, C)
    ch0 = ch.copy()
    ep = ctx.track(d_if.ptr, 0, n, ch, 1, closed_loop=False)[:, 0]
    for i in range(C):
        pad = S.padded_code(system, int(ids[i]))
        sums, blk, pos, rc, rcar = S.correlate(IF, s, pad, int(ch0["pos"][i]),
                                               float(ch0["rem_code"][i]),
                                               float(ch0["rem_carr"][i]),
                                               float(ch0["code_freq"][i]),
                                               float(ch0["carr_freq"][i]))
        assert ep["status"][i] == 0 and ep["blksize"][i] == blk
        assert ch["pos"][i] == pos and ch["rem_code"][i] == rc and ch["rem_carr"][i] == rcar
        got = np.array([ep[f][i] for f in SUMS])
        assert _close(got, sums).all(), (i, got, sums)


def _glonass_scene(gc, n_ms, fs=FS):
    rng = np.random.default_rng(5)
    fchs = np.arange(-7, 7)
    cps = rng.uniform(0, 511, 14)
    dops = rng.uniform(-3000, 3000, 14)
    sigs = [dict(system=1, fch=int(k), code_phase=float(c), doppler=float(d), cn0=48.0,
                 data_bits=1) for k, c, d in zip(fchs, cps, dops)]
    IF = gc.ifgen(int(fs * (n_ms + 3) / 1000), sigs, fs=fs, if_glo=1e6, seed=77)
    acq = 1e6 + 0.5625e6 * fchs + dops + rng.uniform(-15, 15, 14)
    starts = [_glo_start(c, fs) for c in cps]
    return IF, fchs, starts, acq


@pytest.mark.parametrize("fs", RATES)
def test_config4_glonass_14_fch_closed_loop(gpu, fs):
    """BASELINE config 4: 14 FDMA channels, 511-chip ST code, fp64 loop on the GPU
    (at 16.368 Msps too, the rate SURVEY 8(d) states for config 4)."""
    gc = gpu
    n_ms = 150
    IF, fchs, starts, acq = _glonass_scene(gc, n_ms, fs)
    d_if = gc.DevBuf.from_array(IF)
    ctx = gc.SgtCtx(1, samplingFreq=fs)
    ch = ctx.init_chans(fchs, starts, acq)
    ep = ctx.track(d_if.ptr, 0, len(IF) // 2, ch, n_ms, closed_loop=True)
    s = S.settings(1, samplingFreq=fs)
    for i in range(14):
        r = S.track(IF, s, int(fchs[i]), starts[i], float(acq[i]), n_ms)
        assert (ep["status"][i] == 0).all()
        assert (ep["blksize"][i] == r["blksize"]).all()
        for f in S.FIELDS:
            ok = _close(ep[f][i], r[f], rtol=1e-6, atol=1e-6)
            assert ok.all(), (i, f, np.flatnonzero(~ok)[:5], ep[f][i][~ok][:3], r[f][~ok][:3])
    # the loops locked: carrier on the planted frequency within a few Hz
    tail = ep[:, 100:]
    assert (np.median(np.abs(tail["I_P"]), 1) > 3 * np.median(np.abs(tail["Q_P"]), 1)).all()


def test_gps_closed_loop_and_multi_record(gpu):
    """Two records (streams) x 4 PRNs each, GPS C/A tracking.sci loop."""
    gc = gpu
    n_ms = 80
    recs, chans, meta = [], [], []
    for rec in range(2):
        prns = [3 + rec, 9 + rec, 17 + rec, 30 + rec]
        rng = np.random.default_rng(40 + rec)
        cps = rng.uniform(0, 1023, 4)
        dops = rng.uniform(-4000, 4000, 4)
        sigs = [dict(system=0, prn=p, code_phase=float(c), doppler=float(d), cn0=47.0,
                     data_bits=1) for p, c, d in zip(prns, cps, dops)]
        IF = gc.ifgen(int(FS * (n_ms + 2) / 1000), sigs, fs=FS, seed=90 + rec)
        recs.append(IF)
        for p, c, d in zip(prns, cps, dops):
            st = int(round((1023 - c) / 1.023e6 * FS)) + 1
            meta.append((rec, p, st, 2.42e6 + d + 7.0))
    stride = len(recs[0])
    allif = np.concatenate(recs)
    d_if = gc.DevBuf.from_array(allif)
    ctx = gc.SgtCtx(0)
    ch = ctx.init_chans([m[1] for m in meta], [m[2] for m in meta], [m[3] for m in meta],
                        streams=[m[0] for m in meta])
    ep = ctx.track(d_if.ptr, stride, stride // 2, ch, n_ms, closed_loop=True)
    s = S.settings(0)
    for i, (rec, p, st, f0) in enumerate(meta):
        r = S.track(recs[rec], s, p, st, f0, n_ms)
        assert (ep["blksize"][i] == r["blksize"]).all()
        for f in S.FIELDS:
            assert _close(ep[f][i], r[f]).all(), (i, f)


def test_out_of_data_stops_like_tracking_sci(gpu):
    gc = gpu
    IF, fchs, starts, acq = _glonass_scene(gc, 10)
    n = len(IF) // 2
    d_if = gc.DevBuf.from_array(IF)
    ctx = gc.SgtCtx(1)
    ch = ctx.init_chans(fchs[:3], starts[:3], acq[:3])
    ep = ctx.track(d_if.ptr, 0, n, ch, 40, closed_loop=True)
    s = S.settings(1)
    for i in range(3):
        r = S.track(IF, s, int(fchs[i]), starts[i], float(acq[i]), 40)
        k = len(r["I_P"])
        assert k < 40
        assert (ep["status"][i][:k] == 0).all() and (ep["status"][i][k:] == 1).all()
        assert ch["status"][i] == 1 and ch["n_epochs"][i] == k


@pytest.mark.parametrize("reps", [40, 80])
def test_many_channels_launch_shape(gpu, reps):
    """>= 1024 channels switch to one wave per channel: the same closed-loop
    results as the 14-channel (256-thread) launch."""
    gc = gpu
    IF, fchs, starts, acq = _glonass_scene(gc, 4)
    d_if = gc.DevBuf.from_array(IF)
    ctx = gc.SgtCtx(1)
    ch14 = ctx.init_chans(fchs, starts, acq)
    big = np.tile(ch14, reps)                     # 560 / 1120 channels
    small = ch14.copy()
    e_big = ctx.track(d_if.ptr, 0, len(IF) // 2, big, 3, closed_loop=True)
    e_small = ctx.track(d_if.ptr, 0, len(IF) // 2, small, 3, closed_loop=True)
    # The shapes rotate the carrier by T*kC samples per chunk pass (T = 64 / 256
    # threads), from differently rounded fp64 angles of ~2.4e3 rad (ulp 4.5e-13):
    # the phases drift apart by ~1e-12 rad per pass, ~1e-11 relative per epoch.
    for f in S.FIELDS:
        a = e_big[f].reshape(reps, 14, 3)
        assert _close(a, np.broadcast_to(e_small[f], a.shape), rtol=1e-10, atol=1e-8).all(), f
    assert (e_big["blksize"].reshape(reps, 14, 3) == e_small["blksize"]).all()
