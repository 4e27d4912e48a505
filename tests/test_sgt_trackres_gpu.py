"""GPU: sgt.hip's loop half against the reference's recorded tracking runs.

The six recorded sums of SCI/GLONASS/L1/trackingResults.dat and
L2/trackingResults.dat (1500 epochs each, tests/golden/sgt_trackres.npz) drive
`gnsscorr_sgt_replay`, which runs the same device epoch-end code
(`sgt_epoch_end` in csrc/sgt.hip) as the closed-loop tracker: blksize /
remCodePhase chain (tracking.sci:248-302), FLL-assisted PLL (:329-351), DLL
(:353-375), absoluteSample (:379) and codeFreq without aiding (:366), the
variants the record shows.  Tolerances: tests/trackres_fixture.py.  The
tracker itself runs the variants against the oracle on a planted scene.
"""
import numpy as np
import pytest

import sgt_oracle as S
import trackres_fixture as TR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def z():
    return TR.load()


def _ctx(gc, st, **over):
    return gc.SgtCtx(1, **{**TR.scilab_settings(st), **over})


@pytest.mark.parametrize("run", TR.RUNS)
def test_gpu_loop_replays_the_recorded_run(gpu, z, run):
    gc = gpu
    st, fch, acq_freq, code_phase, skip, sums = TR.run_inputs(z, run)
    ctx = _ctx(gc, st)
    ch = ctx.init_chans([fch], [code_phase], [acq_freq], skip=skip)
    ep = ctx.replay(ch, sums[None])[0]
    assert (ep["status"] == 0).all()
    TR.check_against_record(z, run, ep, ep["blksize"])
    # the sums pass through unchanged into the record
    for k in TR.SUMS:
        np.testing.assert_array_equal(ep[k], z[f"{run}_{k}"])
    # and the channel state carries on: pos is the last absoluteSample (mtell form)
    assert ch["pos"][0] == z[f"{run}_absoluteSample"][-1] and ch["n_epochs"][0] == 1500


def test_gpu_replay_many_channels_and_split_calls(gpu, z):
    """Both runs x 64 channels in one launch, and the same in two calls of 700 +
    800 epochs: identical records (the state carries across calls)."""
    gc = gpu
    st, fch, acq_freq, code_phase, skip, _ = TR.run_inputs(z, "L1")
    ctx = _ctx(gc, st)
    sums = np.stack([TR.run_inputs(z, r)[5] for r in TR.RUNS] * 32)
    ch = ctx.init_chans([fch] * 64, [code_phase] * 64, [acq_freq] * 64, skip=skip)
    ch2 = ch.copy()
    ep = ctx.replay(ch, sums)
    a = ctx.replay(ch2, sums[:, :700])
    b = ctx.replay(ch2, sums[:, 700:])
    assert np.array_equal(np.concatenate([a, b], 1).view(np.uint8), ep.view(np.uint8))
    assert np.array_equal(ch.view(np.uint8), ch2.view(np.uint8))
    TR.check_against_record(z, "L1", ep[0], ep["blksize"][0])


def test_gpu_replay_equals_oracle_replay_bit_for_bit_on_exact_fields(gpu, z):
    gc = gpu
    st, fch, acq_freq, code_phase, skip, sums = TR.run_inputs(z, "L2")
    ctx = _ctx(gc, st)
    ch = ctx.init_chans([fch], [code_phase], [acq_freq], skip=skip)
    ep = ctx.replay(ch, sums[None])[0]
    r = S.replay(sums, S.settings(1, **TR.scilab_settings(st)), fch, code_phase, acq_freq,
                 skip=skip)
    np.testing.assert_array_equal(ep["blksize"], r["blksize"])
    for k in TR.EXACT:
        np.testing.assert_array_equal(ep[k], r[k])


@pytest.mark.parametrize("variant", [(1, 1), (0, 1), (1, 0)])
def test_tracker_runs_the_variants_like_the_oracle(gpu, variant):
    """The closed-loop tracker with the record's variants (and each alone) on a
    planted GLONASS scene against the oracle: blksize exact, fields within 1e-6."""
    gc = gpu
    cv, av = variant
    fs, n_ms = 16e6, 60
    rng = np.random.default_rng(9)
    fchs = np.array([-4, 0, 4, 6])
    cps = rng.uniform(0, 511, 4)
    dops = rng.uniform(-2000, 2000, 4)
    sigs = [dict(system=1, fch=int(k), code_phase=float(c), doppler=float(d), cn0=48.0,
                 data_bits=1) for k, c, d in zip(fchs, cps, dops)]
    IF = gc.ifgen(int(fs * (n_ms + 3) / 1000), sigs, fs=fs, if_glo=1e6, seed=12)
    acq = 1e6 + 0.5625e6 * fchs + dops + rng.uniform(-15, 15, 4)
    starts = [int(round((511 - c) / 0.511e6 * fs)) + 1 for c in cps]
    d_if = gc.DevBuf.from_array(IF)
    kw = dict(codeNcoVariant=cv, absSampleVariant=av, dllCorrelatorSpacing=0.5,
              dllNoiseBandwidth=2.0)
    ctx = gc.SgtCtx(1, samplingFreq=fs, **kw)
    ch = ctx.init_chans(fchs, starts, acq)
    ep = ctx.track(d_if.ptr, 0, len(IF) // 2, ch, n_ms, closed_loop=True)
    s = S.settings(1, samplingFreq=fs, **kw)
    for i in range(4):
        r = S.track(IF, s, int(fchs[i]), starts[i], float(acq[i]), n_ms)
        assert (ep["blksize"][i] == r["blksize"]).all()
        for f in S.FIELDS:
            a, b = ep[f][i], r[f]
            assert (np.abs(a - b) <= 1e-6 * np.abs(b) + 1e-6).all(), (i, f)
        if av == 1:
            assert (ep["absoluteSample"][i] == np.round(ep["absoluteSample"][i])).all()
