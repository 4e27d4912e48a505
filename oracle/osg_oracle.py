"""oracle/osg_oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes drivers for
  * liboracle.so        our scalar C restatement of Sim_GP2021_int (osg_corr.c)
  * _ref/libosg_ref.so  the reference correlator.c + gp2021.c + osgpsisr.c
                        compiled from /root/reference (present only where the
                        reference is; never on the GPU box unless prebuilt)

Both expose the same small interface (init / register writes / sim / register
reads / channel state) so tests can run one command schedule through either
and compare every REG_read word and the internal NCO state.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libosg_ref.so")
REF_SRC = ("/root/reference/trunk/GNSS_SOFTWARE_RECEIVERS/POSTPROCESSING_RECEIVERS/"
           "osgnss_next_step/src")


def build(ref: bool = True) -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    if ref and os.path.isdir(REF_SRC):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def have_ref() -> bool:
    return os.path.exists(REF_SO)


class OracleOSG:
    """Our C restatement (osg_corr.c), one emulated GP2021 instance."""

    def __init__(self, n_channels=12, use_iq=True, samp_rate=16.0e6, tic_period=0.0):
        L = C.CDLL(ORACLE_SO)
        L.osgo_sizeof.restype = C.c_int
        L.osgo_init.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double]
        L.osgo_sim.argtypes = [C.c_void_p, C.c_void_p, C.c_long]
        for f in ("osgo_ch_cntl", "osgo_ch_code_slew"):
            getattr(L, f).argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.osgo_ch_epoch_load.argtypes = [C.c_void_p, C.c_int, C.c_uint]
        L.osgo_ch_carrier.argtypes = [C.c_void_p, C.c_int, C.c_long]
        L.osgo_ch_code.argtypes = [C.c_void_p, C.c_int, C.c_long]
        L.osgo_table_bytes.restype = C.c_int
        L.osgo_table_image.argtypes = [C.c_void_p]
        L.osgo_bench.restype = C.c_double
        L.osgo_bench.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_long, C.c_int, C.c_int,
                                 C.c_long, C.c_long, C.c_int]
        self.L = L
        self.buf = C.create_string_buffer(L.osgo_sizeof())
        self.p = C.cast(self.buf, C.c_void_p)
        self.n_channels = n_channels
        L.osgo_init(self.p, n_channels, int(use_iq), samp_rate, tic_period)
        self._st = self._views()

    def _views(self):
        raw = np.frombuffer(self.buf, dtype=np.uint8)
        MAXC = 16
        off = 0
        off += 4 + 4          # n_channels, use_iq
        off += 8 + 8          # tic, tic_ref
        ms = raw[off:off + 4 * MAXC].view(np.int32); off += 4 * MAXC
        bit = raw[off:off + 4 * MAXC].view(np.int32); off += 4 * MAXC
        cp = raw[off:off + 4 * MAXC].view(np.uint32); off += 4 * MAXC
        cc = raw[off:off + 4 * MAXC].view(np.uint32); off += 4 * MAXC
        kp = raw[off:off + 4 * MAXC].view(np.uint32); off += 4 * MAXC
        hc = raw[off:off + 2 * MAXC].view(np.uint16); off += 2 * MAXC
        acc = raw[off:off + 24 * MAXC].view(np.int32).reshape(MAXC, 6); off += 24 * MAXC
        rr = raw[off:off + 1024].view(np.int32); off += 1024
        rw = raw[off:off + 1024].view(np.int32); off += 1024
        return dict(ms=ms, bit=bit, carrier_phase=cp, carrier_cycle=cc, code_phase=kp,
                    half_chip=hc, acc=acc, REG_read=rr, REG_write=rw)

    @property
    def REG_read(self):
        return self._st["REG_read"]

    @property
    def REG_write(self):
        return self._st["REG_write"]

    def ch_cntl(self, ch, prn): self.L.osgo_ch_cntl(self.p, ch, prn)
    def ch_carrier(self, ch, f): self.L.osgo_ch_carrier(self.p, ch, f)
    def ch_code(self, ch, f): self.L.osgo_ch_code(self.p, ch, f)
    def ch_code_slew(self, ch, s): self.L.osgo_ch_code_slew(self.p, ch, s)
    def ch_epoch_load(self, ch, d): self.L.osgo_ch_epoch_load(self.p, ch, d)

    def sim(self, IF: np.ndarray, nsamp: int):
        IF = np.ascontiguousarray(IF, np.int8)
        self.L.osgo_sim(self.p, IF.ctypes.data, nsamp)

    def sim_dumps(self, IF: np.ndarray, nsamp: int, cap: int = 4096) -> np.ndarray:
        """sim() that also returns EVERY dump of the call, [n, 7] int32
        {ch, IL, QL, IP, QP, IE, QE} in sample order (REG_read keeps the last)."""
        log = np.zeros((cap, 7), np.int32)
        self.L.osgo_dump_log.argtypes = [C.c_void_p, C.c_int]
        self.L.osgo_dump_count.restype = C.c_int
        self.L.osgo_dump_log(log.ctypes.data, cap)
        try:
            self.sim(IF, nsamp)
            n = self.L.osgo_dump_count()
        finally:
            self.L.osgo_dump_log(None, 0)
        return log[:n].copy()

    def chan_state(self):
        s = self._st
        n = self.n_channels
        return dict(carrier_phase=s["carrier_phase"][:n].copy(),
                    carrier_cycle=s["carrier_cycle"][:n].copy(),
                    code_phase=s["code_phase"][:n].copy(),
                    half_chip=s["half_chip"][:n].astype(np.uint32),
                    acc=s["acc"][:n].copy(), ms=s["ms"][:n].copy(), bit=s["bit"][:n].copy())

    def table_image(self) -> np.ndarray:
        out = np.empty(self.L.osgo_table_bytes(), np.int8)
        self.L.osgo_table_image(out.ctypes.data)
        return out


class RefOSG:
    """The reference correlator.c/gp2021.c compiled from /root/reference.

    The reference keeps state in process-global variables, so there is one
    instance per process (re-initialised by correlator_init)."""

    _L = None

    def __init__(self, n_channels=12, tic_period=0.0):
        if RefOSG._L is None:
            L = C.CDLL(REF_SO)
            L.correlator_init.argtypes = [C.c_double]
            L.Sim_GP2021_int.argtypes = [C.c_void_p, C.c_long]
            for f in ("ch_cntl", "ch_code_slew"):
                getattr(L, f).argtypes = [C.c_int, C.c_int]
            L.ch_epoch_load.argtypes = [C.c_int, C.c_uint]
            L.ch_carrier.argtypes = [C.c_int, C.c_long]
            L.ch_code.argtypes = [C.c_int, C.c_long]
            RefOSG._L = L
        L = RefOSG._L
        self.L = L
        assert n_channels == 12, "reference N_CHANNELS is a compile-time 12"
        self.n_channels = 12
        self.rr = np.ctypeslib.as_array((C.c_int * 256).in_dll(L, "REG_read"))
        self.rw = np.ctypeslib.as_array((C.c_int * 256).in_dll(L, "REG_write"))
        # a fresh process-global state: the reference only zeroes gpchan
        self.rr[:] = 0
        self.rw[:] = 0
        for name in ("ms_counter", "bit_counter"):
            pass  # file statics: not reachable, start at zero in a fresh process
        L.correlator_init(tic_period)
        self._gp = (C.c_uint8 * (40 * 12)).in_dll(L, "gpchan")

    @property
    def REG_read(self):
        return self.rr

    @property
    def REG_write(self):
        return self.rw

    def ch_cntl(self, ch, prn): self.L.ch_cntl(ch, prn)
    def ch_carrier(self, ch, f): self.L.ch_carrier(ch, f)
    def ch_code(self, ch, f): self.L.ch_code(ch, f)
    def ch_code_slew(self, ch, s): self.L.ch_code_slew(ch, s)
    def ch_epoch_load(self, ch, d): self.L.ch_epoch_load(ch, d)

    def sim(self, IF: np.ndarray, nsamp: int):
        IF = np.ascontiguousarray(IF, np.int8)
        self.L.Sim_GP2021_int(IF.ctypes.data, nsamp)

    def chan_state(self):
        raw = np.frombuffer(self._gp, dtype=np.uint8).reshape(12, 40)
        u = raw.view(np.uint32).reshape(12, 10)
        return dict(carrier_phase=u[:, 0].copy(), carrier_cycle=u[:, 1].copy(),
                    code_phase=u[:, 2].copy(),
                    half_chip=(u[:, 3] & 0xFFFF).astype(np.uint32),
                    # struct order i_prompt,q_prompt,i_late,q_late,i_early,q_early
                    # (correlator.c:41-46) -> REG_read order IL,QL,IP,QP,IE,QE
                    acc=u[:, 4:10].view(np.int32)[:, [2, 3, 0, 1, 4, 5]].copy())


def osg_words(fs: float, gps_if: float = 2.42e6, mult: float = 5.0, cbits: int = 30,
              kbits: int = 29):
    """correlator_init's reference words (correlator.c:110-121) for a sample rate."""
    cdelta = mult * fs / 2.0 ** cbits
    kdelta = mult * fs / 2.0 ** kbits
    return dict(carrier_ref=int(gps_if / cdelta), code_ref=int(1023000 / kdelta),
                d_freq=int(1000 / cdelta), carrier_delta=cdelta, code_delta=kdelta)
