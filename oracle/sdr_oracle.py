"""oracle/sdr_oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes views of
  * OracleSDR: our C restatement of the GPS-SDR int16 strong acquisition
    (oracle/sdr_acq.c, built into liboracle.so), and
  * RefSDR: the reference primitives compiled from their own sources with
    -DNO_SIMD (oracle/_ref/libsdr_ref.so; only where /root/reference exists),
plus a deterministic input generator for the 2.048 Msps CPX buffer the
acquisition consumes (SDR/includes/defines.h:150-151, IF 38.4 kHz signaldef.h:34).
Only tests/, smoke() and bench.py's cpu_baseline use this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsdr_ref.so")
N = 2048
FS = 2048000.0
IF_SDR = 38400.0
RESULT = np.dtype([("sv", "<i4"), ("code_phase", "<i4"), ("doppler", "<i4"),
                   ("magnitude", "<u4"), ("success", "<i4"), ("row", "<i4")])
R1 = np.zeros(16, np.int32)
ROWS = 1240            # baseband_rows (acquisition.cpp:107-110)
R2 = np.array([0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 1], np.int32)


def _p(a):
    return a.ctypes.data


def have_ref() -> bool:
    return os.path.exists(REF_SO)


class OracleSDR:
    def __init__(self):
        L = C.CDLL(ORACLE_SO)
        P, I, D = C.c_void_p, C.c_int, C.c_double
        L.sdro_sine_gen.argtypes = [P, D, D, I]
        L.sdro_twiddles.argtypes = [I, P, P]
        L.sdro_fft.argtypes = [P, I, P, P]
        L.sdro_cmulsc.argtypes = [P, P, P, I, I, I]
        L.sdro_cmag_max.argtypes = [P, I, P, P]
        L.sdro_prep_if.argtypes = [P, D, I, P]
        L.sdro_acq_strong.argtypes = [P, P, I, I, I, I]
        L.sdro_acq_strong.restype = _Res
        L.sdro_prn_codes.argtypes = [P]
        L.sdro_prep_rows.argtypes = [P, I, D, I, P]
        L.sdro_acq_medium.argtypes = [P, P, I, I, I, I]
        L.sdro_acq_medium.restype = _Res
        L.sdro_acq_weak.argtypes = [P, P, I, I, I, I]
        L.sdro_acq_weak.restype = _Res
        L.sdro_weak_shift.argtypes = [I, I, I]
        L.sdro_weak_shift.restype = I
        L.orc_gn3s_block.argtypes = [P, P, C.c_uint32, P, P]
        L.orc_downsample.argtypes = [P, P, D, D, I]
        L.orc_downsample.restype = I
        self.L = L

    def gn3s(self, samples, phase=0, step=2557223528):
        """Read_GN3S + Resample_GN3S over consecutive 5-ms blocks of 20000 bytes
        (gps_source.cpp:684-767, :933-943); returns (out [n*10240, 2] int16, phase)."""
        b = np.ascontiguousarray(samples, np.uint8).reshape(-1, 20000)
        out = np.zeros((b.shape[0] * 10240, 2), np.int16)
        ph = C.c_uint32(phase)
        for k in range(b.shape[0]):
            blk = np.ascontiguousarray(b[k])
            o = out[k * 10240:(k + 1) * 10240]
            self.L.orc_gn3s_block(_p(blk), C.byref(ph), step, _p(o), None)
        return out, ph.value

    def downsample(self, src, fdest, fsource):
        """downsample() (misc.cpp:174-197) of CPX src [n, 2] int16."""
        src = np.ascontiguousarray(src, np.int16)
        out = np.zeros_like(src)
        k = self.L.orc_downsample(_p(out), _p(src), fdest, fsource, src.shape[0])
        return out[:k].copy()

    def sine_gen(self, f, n=N, fs=FS):
        out = np.zeros((n, 2), np.int16)
        self.L.sdro_sine_gen(_p(out), f, fs, n)
        return out

    def fft(self, x, inverse=False, scale=None):
        x = np.ascontiguousarray(x, np.int16).copy()
        n = x.shape[0]
        w = np.zeros((n // 2, 4), np.int16)
        iw = np.zeros((n // 2, 4), np.int16)
        self.L.sdro_twiddles(n, _p(w), _p(iw))
        sc = np.ascontiguousarray(R1 if scale is None else scale, np.int32)
        self.L.sdro_fft(_p(x), n, _p(iw if inverse else w), _p(sc))
        return x

    def cmulsc(self, a, b, shift, saturate=False):
        a = np.ascontiguousarray(a, np.int16)
        b = np.ascontiguousarray(b, np.int16)
        c = np.zeros_like(a)
        self.L.sdro_cmulsc(_p(a), _p(b), _p(c), a.shape[0], shift, int(saturate))
        return c

    def cmag_max(self, a):
        a = np.ascontiguousarray(a, np.int16)
        i, m = C.c_int32(), C.c_int32()
        self.L.sdro_cmag_max(_p(a), a.shape[0], C.byref(i), C.byref(m))
        return i.value, m.value

    def prep_if(self, buff, fif=IF_SDR, saturate=False):
        buff = np.ascontiguousarray(buff, np.int16)
        rows = np.zeros((4, N, 2), np.int16)
        self.L.sdro_prep_if(_p(buff), fif, int(saturate), _p(rows))
        return rows

    def acq_strong(self, buff, codes, svs, doppmin=-15000, doppmax=15000, fif=IF_SDR,
                   saturate=False):
        rows = self.prep_if(buff, fif, saturate)
        out = np.zeros(len(svs), RESULT)
        for k, sv in enumerate(svs):
            code = np.ascontiguousarray(codes[sv], np.int16)
            r = self.L.sdro_acq_strong(_p(rows), _p(code), int(sv), doppmin, doppmax,
                                       int(saturate))
            out[k] = (r.sv, r.code_phase, r.doppler, r.magnitude, r.success, r.row)
        return out

    def prn_codes(self):
        out = np.zeros((51, N, 2), np.int16)
        self.L.sdro_prn_codes(_p(out))
        return out

    # -- medium / weak: an Acquisition object's persistent baseband_rows store
    def new_rows(self):
        return np.zeros((ROWS, N, 2), np.int16)

    def prep_rows(self, rows, buff, ms, fif=IF_SDR, saturate=False):
        buff = np.ascontiguousarray(buff, np.int16).reshape(-1, 2)
        assert buff.shape[0] >= ms * N and rows.shape == (ROWS, N, 2)
        self.L.sdro_prep_rows(_p(buff), ms, fif, int(saturate), _p(rows))

    def acq_search(self, kind, rows, codes, svs, doppmin=-15000, doppmax=15000, saturate=False):
        fn = self.L.sdro_acq_medium if kind == "medium" else self.L.sdro_acq_weak
        out = np.zeros(len(svs), RESULT)
        for k, sv in enumerate(svs):
            code = np.ascontiguousarray(codes[sv], np.int16)
            r = fn(_p(rows), _p(code), int(sv), doppmin, doppmax, int(saturate))
            out[k] = (r.sv, r.code_phase, r.doppler, r.magnitude, r.success, r.row)
        return out

    def weak_shift(self, i, lcv, lcv2):
        return self.L.sdro_weak_shift(i, lcv, lcv2)


class _Res(C.Structure):
    _fields_ = [("sv", C.c_int32), ("code_phase", C.c_int32), ("doppler", C.c_int32),
                ("magnitude", C.c_uint32), ("success", C.c_int32), ("row", C.c_int32)]


class RefSDR:
    def __init__(self):
        L = C.CDLL(REF_SO)
        P, I, D = C.c_void_p, C.c_int, C.c_double
        L.ref_sdr_sine_gen.argtypes = [P, D, D, I]
        L.ref_sdr_fft.argtypes = [P, I, P, I]
        L.ref_sdr_cmulsc.argtypes = [P, P, P, I, I]
        L.ref_sdr_cmag_max.argtypes = [P, I, P, P]
        L.ref_sdr_prn_codes.restype = C.POINTER(C.c_int16)
        L.ref_sdr_acq_strong.argtypes = [P, D, I, I, I, P]
        L.ref_sdr_code_gen.argtypes = [I, P]
        L.ref_sdr_accum.argtypes = [P, P, P, P, P, I, P]
        L.ref_sdr_downsample.argtypes = [P, P, D, D, I]
        L.ref_sdr_downsample.restype = I
        L.ref_sdr_acq_session.argtypes = [D]
        L.ref_sdr_acq_session.restype = P
        L.ref_sdr_acq_session_free.argtypes = [P]
        L.ref_sdr_acq_prep.argtypes = [P, P, I]
        L.ref_sdr_acq_medium.argtypes = [P, I, I, I, P]
        L.ref_sdr_acq_weak.argtypes = [P, I, I, I, P]
        self.L = L

    def downsample(self, src, fdest, fsource):
        src = np.ascontiguousarray(src, np.int16).copy()
        out = np.zeros_like(src)
        k = self.L.ref_sdr_downsample(_p(out), _p(src), fdest, fsource, src.shape[0])
        return out[:k].copy()

    def sine_gen(self, f, n=N, fs=FS):
        out = np.zeros((n, 2), np.int16)
        self.L.ref_sdr_sine_gen(_p(out), f, fs, n)
        return out

    def fft(self, x, inverse=False, scale=None):
        x = np.ascontiguousarray(x, np.int16).copy()
        sc = np.ascontiguousarray(R1 if scale is None else scale, np.int32)
        self.L.ref_sdr_fft(_p(x), x.shape[0], _p(sc), int(inverse))
        return x

    def cmulsc(self, a, b, shift):
        a = np.ascontiguousarray(a, np.int16).copy()
        b = np.ascontiguousarray(b, np.int16).copy()
        c = np.zeros_like(a)
        self.L.ref_sdr_cmulsc(_p(a), _p(b), _p(c), a.shape[0], shift)
        return c

    def cmag_max(self, a):
        a = np.ascontiguousarray(a, np.int16).copy()
        i, m = C.c_int32(), C.c_int32()
        self.L.ref_sdr_cmag_max(_p(a), a.shape[0], C.byref(i), C.byref(m))
        return i.value, m.value

    def code_gen(self, sv):
        out = np.zeros(1023, np.int16)
        self.L.ref_sdr_code_gen(sv, _p(out))
        return out

    def accum(self, data, sine, e, p, l, samps):
        out = np.zeros(6, np.int32)
        keep = [np.ascontiguousarray(data, np.int16).copy(),
                np.ascontiguousarray(sine, np.int16).copy()] + \
            [np.ascontiguousarray(x, np.int8) for x in (e, p, l)]   # alive during the call
        self.L.ref_sdr_accum(*[_p(k) for k in keep], samps, _p(out))
        return out

    def prn_codes(self):
        p = self.L.ref_sdr_prn_codes()
        return np.ctypeslib.as_array(p, shape=(51 * N * 2,)).copy().reshape(51, N, 2)

    def acq_strong(self, buff, svs, doppmin=-15000, doppmax=15000, fif=IF_SDR):
        buff = np.ascontiguousarray(buff, np.int16)
        out = np.zeros(len(svs), RESULT)
        o = np.zeros(6, np.int32)
        for k, sv in enumerate(svs):
            self.L.ref_sdr_acq_strong(_p(buff), fif, int(sv), doppmin, doppmax, _p(o))
            out[k] = tuple(int(v) for v in o)
        return out


class RefAcqSession:
    """The reference Acquisition object's medium/weak path (doPrepIF +
    doAcqMedium / doAcqWeak over the -DNO_SIMD primitives, sdr_ref_harness.cpp),
    with its baseband_rows member persisting between requests."""

    def __init__(self, ref: RefSDR, fif=IF_SDR):
        self.L = ref.L
        self.h = self.L.ref_sdr_acq_session(fif)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ref_sdr_acq_session_free(self.h)
            self.h = None

    def prep(self, buff, ms):
        buff = np.ascontiguousarray(buff, np.int16).reshape(-1, 2)
        assert buff.shape[0] >= ms * N
        self.L.ref_sdr_acq_prep(self.h, _p(buff), ms)

    def search(self, kind, svs, doppmin=-15000, doppmax=15000):
        fn = self.L.ref_sdr_acq_medium if kind == "medium" else self.L.ref_sdr_acq_weak
        out = np.zeros(len(svs), RESULT)
        o = np.zeros(6, np.int32)
        for k, sv in enumerate(svs):
            fn(self.h, int(sv), doppmin, doppmax, _p(o))
            out[k] = tuple(int(v) for v in o)
        return out


def make_long_buffer(sigs, ms, seed=1, amp_noise=2.0, fif=IF_SDR):
    """ms consecutive 1-ms CPX blocks [ms*2048, 2] of one continuous signal
    (make_buffer over the whole span)."""
    return make_buffer(sigs, n=ms * N, seed=seed, amp_noise=amp_noise, fif=fif)


def ca_chips(prn: int) -> np.ndarray:
    """+-1 C/A chips, code_gen (SDR/accessories/misc.cpp:28-87) form."""
    g1 = np.zeros(1023, np.int8)
    g2 = np.zeros(1023, np.int8)
    r1 = [1] * 10
    r2 = [1] * 10
    for k in range(1023):
        g1[k], g2[k] = r1[0], r2[0]
        f1 = r1[7] ^ r1[0]
        f2 = (r2[8] + r2[7] + r2[4] + r2[2] + r2[1] + r2[0]) & 1
        r1 = r1[1:] + [f1]
        r2 = r2[1:] + [f2]
    delays = [5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470,
              471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862]
    d = 1023 - delays[prn - 1]
    return 2 * (g1 ^ g2[(np.arange(1023) + d) % 1023]).astype(np.int16) - 1


def make_buffer(sigs, n=N, seed=1, amp_noise=2.0, fif=IF_SDR):
    """CPX int16 buffer [n, 2] at 2.048 Msps: planted C/A signals at +(fif+doppler),
    complex Gaussian noise, rounded to small integers (AGC-like levels)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / FS
    z = amp_noise * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    for s in sigs:
        chips = ca_chips(s["prn"])
        cp = (s["code_phase"] + t * 1.023e6 * (1 + s["doppler"] / 1575.42e6)) % 1023
        z += s["amp"] * chips[cp.astype(np.int64)] * np.exp(2j * np.pi * (fif + s["doppler"]) * t)
    out = np.zeros((n, 2), np.int16)
    out[:, 0] = np.clip(np.round(z.real), -127, 127)
    out[:, 1] = np.clip(np.round(z.imag), -127, 127)
    return out


# ---------------------------------------------------------------- tracking correlator
CHAN = np.dtype([("code_phase", "<f8"), ("carrier_phase", "<f8"), ("carrier_phase_prev", "<f8"),
                 ("code_phase_mod", "<f8"), ("carrier_phase_mod", "<f8"), ("code_nco", "<f8"),
                 ("carrier_nco", "<f8"), ("chan", "<u4"), ("sv", "<u4"), ("navigate", "<u4"),
                 ("active", "<u4"), ("count", "<u4"), ("scount", "<u4"), ("epoch_1ms", "<u4"),
                 ("epoch_20ms", "<u4"), ("z_count", "<u4"), ("rollover", "<u4"),
                 ("cbin", "<u4", (3,)), ("sbin", "<u4"), ("coff", "<i4", (3,)), ("soff", "<i4")])
CORR = np.dtype([("i", "<i4", (3,)), ("q", "<i4", (3,))])
ROW, SBINS, CBINS = 4096, 3001, 101


class OracleSdrCorr:
    """Scalar restatement of the GPS-SDR Correlator (oracle/sdr_corr.c)."""

    def __init__(self, saturate=False):
        L = C.CDLL(ORACLE_SO)
        P, I, D = C.c_void_p, C.c_int, C.c_double
        L.sdrc_tables.argtypes = [P, P]
        L.sdrc_code_gen.argtypes = [I, P]
        L.sdrc_accum.argtypes = [P, P, P, P, P, I, I, P]
        L.sdrc_correlate.argtypes = [P, P, I, P, P, I, P, P]
        L.sdrc_init_chan.argtypes = [P, I, I, I, D]
        self.L = L
        self.saturate = int(saturate)
        self.carrier = np.zeros((SBINS, ROW, 2), np.int16)
        self.code = np.zeros((32, CBINS, ROW), np.int8)
        L.sdrc_tables(_p(self.carrier), _p(self.code))
        self._t = (C.c_void_p * 2)(self.carrier.ctypes.data, self.code.ctypes.data)
        self.test_loop = C.cast(L.sdrc_test_loop, C.c_void_p).value

    def code_gen(self, sv):
        out = np.zeros(1023, np.uint8)
        self.L.sdrc_code_gen(sv, _p(out))
        return out

    def accum(self, data, job):
        """One Accum job over flat tables (SDR_JOB-like dict/record); returns CORR record."""
        c = np.zeros(1, CORR)
        sv, sb, so = int(job["sv"]), int(job["sbin"]), int(job["soff"])
        flat_car = self.carrier.reshape(-1, 2)
        flat_code = self.code.reshape(-1)
        sine = np.ascontiguousarray(flat_car[sb * ROW + so:])
        codes = [np.ascontiguousarray(flat_code[(sv * CBINS + int(job["cbin"][k])) * ROW +
                                                int(job["coff"][k]):]) for k in range(3)]
        d = np.ascontiguousarray(data[int(job["data_off"]):])
        self.L.sdrc_accum(_p(d), _p(sine), _p(codes[0]), _p(codes[1]), _p(codes[2]),
                          int(job["samps"]), self.saturate, _p(c))
        return c[0]

    def init_chan(self, sv, cp, dop, since=0.0):
        s = np.zeros(1, CHAN)
        self.L.sdrc_init_chan(_p(s), sv, cp, dop, since)
        return s[0]

    def correlate(self, packet, states, corr, cb=None, user=None):
        packet = np.ascontiguousarray(packet, np.int16)
        self.L.sdrc_correlate(C.byref(self._t), _p(packet), len(states), _p(states), _p(corr),
                              self.saturate, cb if cb is not None else self.test_loop, user)


# ---------------------------------------------------------------- GPS-SDR Channel
REF_CHAN_SO = os.path.join(HERE, "_ref", "libsdr_chan_ref.so")


def have_ref_chan() -> bool:
    return os.path.exists(REF_CHAN_SO)


class RefSdrChannel:
    """The reference Channel object itself (objects/channel.cpp built with
    -DNO_SIMD, oracle/sdr_chan_ref.cpp): Start, Accum per 1-ms correlation,
    state read-back and the subframes it writes to the ephemeris pipe."""

    FB = np.dtype([("carrier_nco", "<f8"), ("code_nco", "<f8"), ("kill", "<u4"),
                   ("reset_1ms", "<u4"), ("reset_20ms", "<u4"), ("set_z_count", "<u4"),
                   ("z_count", "<u4"), ("length", "<u4"), ("navigate", "<u4"), ("pad", "<u4")])
    SUB = np.dtype([("sv", "<i4"), ("subframe", "<i4"), ("word_buff", "<u4", (12,))])

    def __init__(self, chan=0):
        L = C.CDLL(REF_CHAN_SO)
        P, I = C.c_void_p, C.c_int
        L.ref_chan_new.restype = P
        L.ref_chan_new.argtypes = [I]
        L.ref_chan_free.argtypes = [P]
        L.ref_chan_start.argtypes = [P, I, I, I]
        L.ref_chan_accum.argtypes = [P, P, P]
        L.ref_chan_state.argtypes = [P, P]
        L.ref_chan_read_subframes.argtypes = [P, I]
        L.ref_chan_read_subframes.restype = I
        L.ref_chan_parity.argtypes = [C.c_uint32]
        L.ref_chan_parity.restype = I
        self.L = L
        self.h = L.ref_chan_new(chan)
        self.ssize = L.ref_chan_state_size()

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ref_chan_free(self.h)
            self.h = None

    def start(self, sv, doppler, corr_len=1):
        self.L.ref_chan_start(self.h, int(sv), int(doppler), int(corr_len))

    def state(self) -> np.ndarray:
        out = np.zeros(self.ssize, np.uint8)
        self.L.ref_chan_state(self.h, _p(out))
        return out

    def run(self, corr):
        """Accum over corr (n_ms, 6) int32; returns (feedback FB[n_ms], subframes as
        (ms, SUB record) pairs, final state bytes)."""
        corr = np.ascontiguousarray(corr, np.int32)
        fb = np.zeros(len(corr), self.FB)
        subs = []
        buf = np.zeros(64, self.SUB)
        for m in range(len(corr)):
            row = np.ascontiguousarray(corr[m])
            self.L.ref_chan_accum(self.h, _p(row), fb[m:m + 1].ctypes.data)
            n = self.L.ref_chan_read_subframes(_p(buf), 64)
            subs.extend((m, buf[k].copy()) for k in range(n))
        return fb, subs, self.state()

    def parity(self, word: int) -> bool:
        return bool(self.L.ref_chan_parity(word & 0xFFFFFFFF))
