"""GPU parity: the OSGPS channel loops (gpsisr) on the GPU, bit-exact.

Reference: osgnss_next_step/src/isr/osgpsisr.c:360-768 (gpsisr, ch_acq,
ch_confirm, ch_pull_in, ch_track) and gp2021/gp2021.c:75-130 (register words).
(1) One interrupt from random channel states in every state against the
    UNMODIFIED reference gpsisr (oracle/_ref/libosg_ref.so, ref_isr_step):
    every loop field and every register word it writes.
(2) The device-resident closed loop (gnsscorr_track_dev + gnsscorr_osg_isr_dev
    per 512-us call, no host in the loop) against the reference receiver run
    (oracle/_ref/e2e_ref: reference correlator.c + gp2021.c + osgpsisr.c) on the
    same recording: state, NCO frequencies, search counters and accumulators of
    every call.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libosg_ref.so")
E2E_REF = os.path.join(ROOT, "oracle", "_ref", "e2e_ref")
REC = np.dtype([("reg", "<i4", 256), ("state", "<i4", 12), ("carr", "<i8", 12),
                ("code", "<i8", 12), ("nfreq", "<i4", 12), ("codes", "<i4", 12)])
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built")]
FIELDS = ["state", "n_freq", "i_confirm", "n_thresh", "codes", "del_freq", "sign_pos",
          "prev_sign_pos", "sign_count", "ms_count", "ms_set", "search_max_prn_delay",
          "search_max_f", "cn0", "bit", "accum", "prev_accum", "early_mag", "prompt_mag",
          "late_mag", "cross", "dot", "carr_error", "old_carr_error", "freq_error", "carr_nco",
          "old_carr_nco", "carr_freq", "carr_freq_basis", "code_error", "old_code_error",
          "code_freq", "code_freq_basis", "code_nco", "old_code_nco", "ch_time", "carrier_freq",
          "carrier_cold_corr", "ms_sign"]


def _ref():
    L = C.CDLL(REF_SO)
    L.ref_isr_set_chan.argtypes = [C.c_int, C.c_void_p]
    L.ref_isr_get_chan.argtypes = [C.c_int, C.c_void_p]
    L.ref_isr_step.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
    L.ref_isr_constants.argtypes = [C.c_void_p]
    out = (C.c_long * 8)()
    L.ref_isr_constants(out)      # loop coefficients + correlator_init words
    return L


def _random_loops(gc, rng, n, cfg):
    lo = np.zeros(n, gc.OSG_LOOP)
    lo["state"] = rng.integers(1, 5, n)
    lo["n_freq"] = rng.integers(-6, 7, n)
    lo["i_confirm"] = rng.integers(0, 4, n)
    lo["n_thresh"] = rng.integers(0, 3, n)
    lo["codes"] = np.where(rng.random(n) < 0.3, 2044, rng.integers(0, 2045, n))
    lo["del_freq"] = rng.integers(-6, 7, n)
    lo["sign_pos"] = rng.integers(0, 3000, n)
    lo["prev_sign_pos"] = rng.integers(0, 3000, n)
    lo["sign_count"] = rng.integers(25, 35, n)
    lo["ms_count"] = rng.integers(0, 20, n)
    lo["ms_set"] = rng.integers(0, 2, n)
    lo["search_max_prn_delay"] = 2045
    lo["search_max_f"] = 5
    small = rng.random((n, 6)) < 0.4
    big = rng.integers(-32768, 32768, (n, 6))
    lo["accum"] = np.where(small, rng.integers(-3, 4, (n, 6)), big)
    lo["prev_accum"] = rng.integers(-3000, 3001, (n, 6))
    for f in ("early_mag", "prompt_mag", "late_mag"):
        lo[f] = rng.integers(0, 100000, n)
    for f in ("carr_error", "old_carr_error", "freq_error", "code_error", "old_code_error"):
        lo[f] = rng.integers(-40000, 40000, n)
    for f in ("carr_nco", "old_carr_nco", "code_nco", "old_code_nco"):
        lo[f] = rng.integers(-200000, 200000, n)
    lo["carrier_freq"] = cfg.carrier_ref + rng.integers(-80000, 80000, n)
    lo["carr_freq_basis"] = lo["carrier_freq"]
    lo["code_freq_basis"] = cfg.code_ref
    lo["ch_time"] = np.where(rng.random(n) < 0.2, 2999, rng.integers(0, 3000, n))
    lo["ms_sign"] = rng.integers(0, 1 << 62, n, dtype=np.int64).astype(np.uint64)
    lo["ms_sign"][::5] = 0xFFFFF
    lo["ms_sign"][1::5] = 0
    return lo


def _regs_from_cmds(cmds):
    regs = np.zeros(256, np.int32)
    for ch, c in enumerate(cmds):
        reg = ch << 3
        regs[reg] = c["prn"]
        regs[reg + 3], regs[reg + 4] = int(c["carrier_incr"]) >> 16, int(c["carrier_incr"]) & 0xFFFF
        regs[reg + 5], regs[reg + 6] = int(c["code_incr"]) >> 16, int(c["code_incr"]) & 0xFFFF
        regs[reg + 7] = c["epoch_load"]
        regs[reg + 0x84] = c["slew"]
    return regs


def test_isr_step_vs_reference(gpu):
    L = _ref()
    cfg = gpu.osg_loop_cfg()
    rng = np.random.default_rng(17)
    n = 12
    trk = gpu.TrackCtx(n, iq=True, samp_rate=16.0e6)
    for it in range(300):
        loops = _random_loops(gpu, rng, n, cfg)
        _, cmds = gpu.osg_loop_reset(cfg, rng.integers(1, 33, n))
        cmds["epoch_load"] = -1
        cmds["slew"] = 0
        res = np.zeros(n, gpu.TRACK_RESULT)
        dumped = rng.random(n) < 0.85
        res["n_dumps"] = dumped.astype(np.int32)
        res["dump"] = np.where(rng.random((n, 6)) < 0.1, 0,
                               rng.integers(-(1 << 20), 1 << 20, (n, 6)))
        # reference: same registers, same REG_read words, one gpsisr()
        for ch in range(n):
            L.ref_isr_set_chan(ch, loops[ch:ch + 1].ctypes.data)
        regs = _regs_from_cmds(cmds)
        mask = int(sum(1 << ch for ch in range(n) if dumped[ch]))
        dumps = np.ascontiguousarray(res["dump"], np.int32)
        L.ref_isr_step(mask, dumps.ctypes.data, regs.ctypes.data)
        want = np.zeros(n, gpu.OSG_LOOP)
        for ch in range(n):
            L.ref_isr_get_chan(ch, want[ch:ch + 1].ctypes.data)
        # GPU
        d_l, d_c, d_r = (gpu.DevBuf.from_array(a) for a in (loops, cmds, res))
        gpu.osg_isr_dev(trk, cfg, n, d_l.ptr, d_c.ptr, d_r.ptr)
        trk.sync()
        got = d_l.download(np.uint8).view(gpu.OSG_LOOP)
        gcm = d_c.download(np.uint8).view(gpu.NCO_CMD)
        for f in FIELDS:
            assert np.array_equal(got[f], want[f]), (it, f, got[f], want[f])
        for ch in range(n):
            reg = ch << 3
            assert gcm[ch]["carrier_incr"] == ((regs[reg + 3] & 0xFFFF) << 16) + (regs[reg + 4] & 0xFFFF)
            assert gcm[ch]["code_incr"] == ((regs[reg + 5] & 0xFFFF) << 16) + (regs[reg + 6] & 0xFFFF)
            assert gcm[ch]["slew"] == (regs[reg + 0x84] & 0xFFFF), (it, ch)
            assert gcm[ch]["epoch_load"] == regs[reg + 7], (it, ch)


def _closed_loop(gpu, tmp_path, calls, sigs, prns, seed):
    IF = gpu.ifgen(8192 * calls, sigs, fs=16.0e6, if_gps=2.42e6, seed=seed)
    f_if = tmp_path / "if.bin"
    IF.tofile(f_if)
    tr_path = tmp_path / "ref.trace"
    subprocess.run([E2E_REF, str(f_if), str(tr_path), str(calls)] + [str(p) for p in prns],
                   check=True, timeout=900)
    ref = np.fromfile(tr_path, REC)
    n = 12
    cfg = gpu.osg_loop_cfg()
    allp = list(prns) + [0] * (n - len(prns))
    loops, cmds = gpu.osg_loop_reset(cfg, allp)
    trk = gpu.TrackCtx(n, iq=True, samp_rate=16.0e6, max_nsamp=8192)
    d_if = gpu.DevBuf.from_array(IF)
    d_l, d_c = gpu.DevBuf.from_array(loops), gpu.DevBuf.from_array(cmds)
    d_rh = gpu.DevBuf(calls * n * gpu.TRACK_RESULT.itemsize)
    d_lh = gpu.DevBuf(calls * n * gpu.OSG_LOOP.itemsize)
    gpu.osg_closed_loop_dev(trk, cfg, d_if.ptr, 0, 8192, calls, n, d_l.ptr, d_c.ptr, d_rh.ptr,
                            d_lh.ptr)
    trk.sync()
    rh = d_rh.download(np.uint8).view(gpu.TRACK_RESULT).reshape(calls, n)
    lh = d_lh.download(np.uint8).view(gpu.OSG_LOOP).reshape(calls, n)
    return ref, rh, lh


def _compare(ref, rh, lh, n_active):
    assert (lh["exited"] == 0).all()
    for ch in range(n_active):
        assert np.array_equal(lh["state"][:, ch], ref["state"][:, ch]), ch
        assert np.array_equal(lh["carrier_freq"][:, ch] + lh["carr_freq"][:, ch],
                              ref["carr"][:, ch]), ch
        assert np.array_equal(lh["code_freq"][:, ch], ref["code"][:, ch]), ch
        assert np.array_equal(lh["n_freq"][:, ch], ref["nfreq"][:, ch]), ch
        assert np.array_equal(lh["codes"][:, ch], ref["codes"][:, ch]), ch
        dumped = rh["n_dumps"][:, ch] > 0
        assert np.array_equal(dumped, (ref["reg"][:, 0x82] >> ch) & 1 == 1), ch
        regs = ref["reg"][:, (ch << 3) + 0x84:(ch << 3) + 0x8A]
        assert np.array_equal(rh["dump"][dumped, ch], regs[dumped]), ch


@pytest.mark.skipif(not os.path.exists(E2E_REF), reason="oracle/_ref/e2e_ref not built")
def test_closed_loop_prn27_vs_reference_receiver(gpu, tmp_path):
    sig = [dict(system=0, prn=27, code_phase=1000.0, doppler=300.0, cn0=52.0, data_bits=1)]
    ref, rh, lh = _closed_loop(gpu, tmp_path, 6000, sig, [27], seed=7)
    _compare(ref, rh, lh, 1)
    assert {1, 2, 3} <= set(np.unique(lh["state"][:, 0]).tolist())


@pytest.mark.skipif(not os.path.exists(E2E_REF), reason="oracle/_ref/e2e_ref not built")
def test_closed_loop_twelve_channels_vs_reference_receiver(gpu, tmp_path):
    prns = [3, 7, 11, 14, 17, 19, 21, 24, 27, 28, 31, 32]
    rng = np.random.default_rng(5)
    sigs = [dict(system=0, prn=p, code_phase=float(rng.uniform(0, 1023)),
                 doppler=float(rng.uniform(-400, 400)), cn0=50.0, data_bits=1)
            for p in prns[:8]]
    ref, rh, lh = _closed_loop(gpu, tmp_path, 2000, sigs, prns, seed=11)
    _compare(ref, rh, lh, 12)


def test_fused_closed_loop_equals_two_launches(gpu, monkeypatch):
    """The closed loop with gpsisr fused into the correlator launch (one launch
    per call, osg_stream_kernel) equals the two-launch form (correlator, then
    osg_isr_kernel; GNSSCORR_OSG_FUSED=0) byte for byte: every call's results,
    loop states and the final commands, 96 channels x 400 calls on 8 receivers."""
    calls, n, n_rx = 400, 96, 8
    rng = np.random.default_rng(21)
    recs = []
    for r in range(n_rx):
        prns = rng.choice(np.arange(1, 33), 6, replace=False)
        sigs = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
                     doppler=float(rng.uniform(-400, 400)), cn0=50.0, data_bits=1) for p in prns]
        recs.append(gpu.ifgen(8192 * calls, sigs, fs=16.0e6, if_gps=2.42e6, seed=40 + r))
    stride = len(recs[0]) // 2
    IF = np.concatenate(recs)
    cfg = gpu.osg_loop_cfg()
    prns = rng.integers(1, 33, n)
    out = []
    for fused in ("1", "0"):
        monkeypatch.setenv("GNSSCORR_OSG_FUSED", fused)
        loops, cmds = gpu.osg_loop_reset(cfg, prns)
        cmds["stream"] = np.arange(n) // 12
        trk = gpu.TrackCtx(n, iq=True, samp_rate=16.0e6, max_nsamp=8192)
        d_if = gpu.DevBuf.from_array(IF)
        d_l, d_c = gpu.DevBuf.from_array(loops), gpu.DevBuf.from_array(cmds)
        d_rh = gpu.DevBuf(calls * n * gpu.TRACK_RESULT.itemsize)
        d_lh = gpu.DevBuf(calls * n * gpu.OSG_LOOP.itemsize)
        gpu.osg_closed_loop_dev(trk, cfg, d_if.ptr, stride, 8192, calls, n, d_l.ptr, d_c.ptr,
                                d_rh.ptr, d_lh.ptr)
        trk.sync()
        out.append((d_rh.download(np.uint8), d_lh.download(np.uint8), d_l.download(np.uint8),
                    d_c.download(np.uint8)))
    for a, b, name in zip(out[0], out[1], ("results", "loop history", "loops", "commands")):
        assert np.array_equal(a, b), name
    lh = out[0][1].view(gpu.OSG_LOOP).reshape(calls, n)
    assert (lh["state"][-1] >= 2).sum() >= 8     # some channels went past acquisition
