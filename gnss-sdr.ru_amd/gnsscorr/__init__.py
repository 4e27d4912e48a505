"""gnsscorr -- Python (ctypes) view of libgnsscorr.so, the MI355X GNSS correlator.

This module is plumbing for tests and benchmarks: every computation happens in
the HIP kernels behind the C ABI declared in include/gnsscorr.h.  There is no
CPU fallback -- if the shared library (or a GPU, for compute calls) is
missing, the calls raise.

Two views are provided:

* ``TrackCtx`` / ``AcqCtx``: the batched API (explicit state, many channels).
* ``OSG``: the reference's GP2021 register interface (correlator_init,
  Sim_GP2021_int, REG_read/REG_write + the gp2021.c accessors ch_carrier,
  ch_code, ch_code_slew, ch_cntl, ch_epoch_load, ch_{i,q}_{early,prompt,late},
  accum_status), so host-loop tests read like the reference's own
  osgnss_next_step.c main loop.
"""
from __future__ import annotations

import ctypes as C
import os
import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# GNSSCORR_LIB: an alternative build of the same library (A/B timing in tools/)
LIB_PATH = os.environ.get("GNSSCORR_LIB") or os.path.join(_HERE, "libgnsscorr.so")

# ---------------------------------------------------------------- structs
NCO_CMD = np.dtype([("prn", "<i4"), ("carrier_incr", "<u4"), ("code_incr", "<u4"),
                    ("slew", "<u4"), ("epoch_load", "<i4"), ("stream", "<i4")])
CHAN_STATE = np.dtype([("carrier_phase", "<u4"), ("carrier_cycle", "<u4"),
                       ("code_phase", "<u4"), ("half_chip", "<u4"), ("acc", "<i4", (6,)),
                       ("ms_counter", "<i4"), ("bit_counter", "<i4"), ("msbit_reg", "<i4"),
                       ("pad", "<i4")])
TRACK_RESULT = np.dtype([("n_dumps", "<i4"), ("dump", "<i4", (6,)), ("msbit_reg", "<i4"),
                         ("tic", "<i4"), ("tic_regs", "<i4", (6,)), ("pad", "<i4")])
ACQ_ROW = np.dtype([("peak", "<f8"), ("second", "<f8"), ("argmax", "<i4"), ("block", "<i4")])
ACQ_RESULT = np.dtype([("peak", "<f8"), ("second", "<f8"), ("metric", "<f8"), ("bin", "<i4"),
                       ("code_phase", "<i4"), ("pad", "<i4"), ("pad2", "<i4"),
                       ("carr_freq", "<f8")])
SIG = np.dtype([("system", "<i4"), ("prn", "<i4"), ("fch", "<i4"), ("data_bits", "<i4"),
                ("code_phase", "<f8"), ("doppler", "<f8"), ("cn0", "<f8"),
                ("carr_phase", "<f8")])
assert NCO_CMD.itemsize == 24 and CHAN_STATE.itemsize == 56 and TRACK_RESULT.itemsize == 64
assert ACQ_ROW.itemsize == 24 and ACQ_RESULT.itemsize == 48 and SIG.itemsize == 48

OSG_LOOP = np.dtype([("state", "<i4"), ("n_freq", "<i4"), ("i_confirm", "<i4"),
                     ("n_thresh", "<i4"), ("codes", "<i4"), ("del_freq", "<i4"),
                     ("sign_pos", "<i4"), ("prev_sign_pos", "<i4"), ("sign_count", "<i4"),
                     ("ms_count", "<i4"), ("ms_set", "<i4"), ("search_max_prn_delay", "<i4"),
                     ("search_max_f", "<i4"), ("cn0", "<i4"), ("bit", "<i4"), ("exited", "<i4"),
                     ("accum", "<i2", (6,)), ("prev_accum", "<i2", (6,)),
                     ("early_mag", "<i8"), ("prompt_mag", "<i8"), ("late_mag", "<i8"),
                     ("cross", "<i8"), ("dot", "<i8"), ("carr_error", "<i8"),
                     ("old_carr_error", "<i8"), ("freq_error", "<i8"), ("carr_nco", "<i8"),
                     ("old_carr_nco", "<i8"), ("carr_freq", "<i8"), ("carr_freq_basis", "<i8"),
                     ("code_error", "<i8"), ("old_code_error", "<i8"), ("code_freq", "<i8"),
                     ("code_freq_basis", "<i8"), ("code_nco", "<i8"), ("old_code_nco", "<i8"),
                     ("ch_time", "<i8"), ("carrier_freq", "<i8"), ("carrier_cold_corr", "<i8"),
                     ("ms_sign", "<u8")])
assert OSG_LOOP.itemsize == 264

SGT_CHAN = np.dtype([("code_id", "<i4"), ("stream", "<i4"), ("status", "<i4"),
                     ("n_epochs", "<i4"), ("pos", "<i8"), ("pad", "<i8"),
                     ("rem_code", "<f8"), ("rem_carr", "<f8"), ("code_freq", "<f8"),
                     ("carr_freq", "<f8"), ("carr_freq_basis", "<f8"), ("old_code_nco", "<f8"),
                     ("old_code_error", "<f8"), ("old_carr_nco", "<f8"),
                     ("old_carr_error", "<f8"), ("i1", "<f8"), ("q1", "<f8"), ("pad2", "<f8")])
SGT_EPOCH = np.dtype([("I_E", "<f8"), ("I_P", "<f8"), ("I_L", "<f8"), ("Q_E", "<f8"),
                      ("Q_P", "<f8"), ("Q_L", "<f8"), ("carrFreq", "<f8"), ("codeFreq", "<f8"),
                      ("absoluteSample", "<f8"), ("dllDiscr", "<f8"), ("dllDiscrFilt", "<f8"),
                      ("pllDiscr", "<f8"), ("pllDiscrFilt", "<f8"), ("blksize", "<i4"),
                      ("status", "<i4")])
assert SGT_CHAN.itemsize == 128 and SGT_EPOCH.itemsize == 112
SDR_CHAN = np.dtype([("code_phase", "<f8"), ("carrier_phase", "<f8"),
                     ("carrier_phase_prev", "<f8"), ("code_phase_mod", "<f8"),
                     ("carrier_phase_mod", "<f8"), ("code_nco", "<f8"), ("carrier_nco", "<f8"),
                     ("chan", "<u4"), ("sv", "<u4"), ("navigate", "<u4"), ("active", "<u4"),
                     ("count", "<u4"), ("scount", "<u4"), ("epoch_1ms", "<u4"),
                     ("epoch_20ms", "<u4"), ("z_count", "<u4"), ("rollover", "<u4"),
                     ("cbin", "<u4", (3,)), ("sbin", "<u4"), ("coff", "<i4", (3,)),
                     ("soff", "<i4")])
SDR_CORR = np.dtype([("i", "<i4", (3,)), ("q", "<i4", (3,))])
SDR_JOB = np.dtype([("packet", "<i4"), ("data_off", "<i4"), ("samps", "<i4"), ("sv", "<i4"),
                    ("sbin", "<i4"), ("soff", "<i4"), ("cbin", "<i4", (3,)),
                    ("coff", "<i4", (3,))])
assert SDR_CHAN.itemsize == 128 and SDR_CORR.itemsize == 24 and SDR_JOB.itemsize == 48
# gnsscorr_sdr_channel: the Channel object's state (objects/channel.h:53-132)
_CH_CORE = [("carrier_nco", "<f8"), ("code_nco", "<f8"), ("len", "<i4"), ("count", "<i4"),
            ("state", "<i4"), ("sv", "<i4"), ("chan", "<i4"), ("I", "<i4", (3,)),
            ("Q", "<i4", (3,)), ("P", "<i4", (3,)), ("I_prev", "<i4"), ("Q_prev", "<i4"),
            ("I_avg", "<f4"), ("Q_var", "<f4"), ("P_avg", "<f4"), ("cn0", "<f4"),
            ("bit_lock", "<i4"), ("bit_lock_pend", "<i4"), ("bit_lock_ticks", "<i4"),
            ("I_sum20", "<i4"), ("Q_sum20", "<i4"), ("I_buff", "<i4", (20,)),
            ("Q_buff", "<i4", (20,)), ("P_buff", "<i4", (20,)), ("epoch_20ms", "<i4"),
            ("epoch_1ms", "<i4"), ("best_epoch", "<i4"), ("valid_frame", "<i4", (5,)),
            ("navigate", "<i4"), ("z_lock", "<i4"), ("converged", "<i4"), ("frame_z", "<i4"),
            ("z_count", "<i4"), ("z_count_pend", "<i4"), ("word_buff", "<u4", (12,)),
            ("frame_lock", "<i4"), ("frame_lock_pend", "<i4"), ("bit_number", "<i4"),
            ("subframe", "<i4"), ("freq_lock", "<i4"), ("freq_lock_ticks", "<i4"),
            ("pll", "<f4", (17,)), ("dll", "<f4", (7,))]
# the C structs' trailing alignment padding as named fields: numpy copies
# (copy(), element assignment) skip unnamed padding bytes, which then hold
# whatever np.empty left there and make byte comparisons of copies flaky
SDR_CHANNEL_CORE = np.dtype(_CH_CORE + [("_pad", "<u4")], align=True)
SDR_CHANNEL = np.dtype(_CH_CORE + [("fft_buff", "<u4", (512,)), ("_pad", "<u4")], align=True)
SDR_SUBFRAME = np.dtype([("sv", "<i4"), ("subframe", "<i4"), ("word_buff", "<u4", (12,)),
                         ("chan", "<i4"), ("ms", "<i4")])
SDR_FEEDBACK = np.dtype([("carrier_nco", "<f8"), ("code_nco", "<f8"), ("kill", "<u4"),
                         ("reset_1ms", "<u4"), ("reset_20ms", "<u4"), ("set_z_count", "<u4"),
                         ("z_count", "<u4"), ("length", "<u4"), ("navigate", "<u4"),
                         ("pad", "<u4")])
SDR_DUMP_REC = np.dtype([("packet", "<i4"), ("phase", "<i4"), ("corr", SDR_CORR),
                         ("fb", SDR_FEEDBACK)])
assert SDR_DUMP_REC.itemsize == 80
assert SDR_CHANNEL_CORE.itemsize == 584 and SDR_CHANNEL.itemsize == 2632
assert SDR_SUBFRAME.itemsize == 64 and SDR_FEEDBACK.itemsize == 48
SDR_ACQ_STRONG, SDR_ACQ_MEDIUM, SDR_ACQ_WEAK = 0, 1, 2   # ACQ_TYPE_* (acquisition.cpp:584-599)
SDR_ACQ_MS = {0: 1, 1: 10, 2: 310}                       # ms per request (acquisition.cpp:628-641)
SDR_RESULT = np.dtype([("sv", "<i4"), ("code_phase", "<i4"), ("doppler", "<i4"),
                       ("magnitude", "<u4"), ("success", "<i4"), ("row", "<i4")])

IF_IQ = 1        # GNSSCORR_IF_IQ: interleaved I,Q
IF_PACKED2 = 2   # GNSSCORR_IF_PACKED2: 2-bit codes, 4 elements per byte (GN3S LUT {-3,-1,1,3})
ACQ_BEST_OF_BLOCKS = 0
ACQ_NONCOHERENT = 1
ACQ_F64 = 0      # reference precision (acquisition.sci evaluates in doubles)
ACQ_F32 = 1      # single-precision fast path (n_samples 16368 only)
CODE_GLO_ST = 0  # GNSSCORR_CODE_GLO_ST: the GLONASS ST code id of set_prn_codes


class TrackCfg(C.Structure):
    _fields_ = [("n_channels", C.c_int), ("iq", C.c_int), ("device", C.c_int),
                ("max_nsamp", C.c_int), ("samp_rate", C.c_double), ("tic_period", C.c_double)]


class AcqCfg(C.Structure):
    _fields_ = [("samp_rate", C.c_double), ("n_samples", C.c_int), ("device", C.c_int),
                ("max_freqs", C.c_int), ("max_blocks", C.c_int), ("max_codes", C.c_int),
                ("precision", C.c_int)]


class SgtCfg(C.Structure):
    _fields_ = [("system", C.c_int32), ("file_type", C.c_int32), ("switch_iq", C.c_int32),
                ("code_length", C.c_int32), ("device", C.c_int32), ("max_channels", C.c_int32),
                ("samp_rate", C.c_double), ("code_freq_basis", C.c_double),
                ("if_freq", C.c_double), ("l1_if_step", C.c_double),
                ("glonass_zero_channel", C.c_double), ("dll_spacing", C.c_double),
                ("dll_noise_bw", C.c_double), ("dll_damping", C.c_double),
                ("pll_noise_bw", C.c_double), ("fll_noise_bw", C.c_double),
                ("code_nco_variant", C.c_int32), ("abs_sample_variant", C.c_int32)]


class SdrCorrCfg(C.Structure):
    _fields_ = [("device", C.c_int32), ("saturate", C.c_int32)]


class SdrAcqCfg(C.Structure):
    _fields_ = [("fif", C.c_double), ("device", C.c_int32), ("saturate", C.c_int32)]


# every symbol include/gnsscorr.h + include/gnsscorr_osg.h declare
EXPORTED_FUNCTIONS = [
    "gnsscorr_last_error", "gnsscorr_version", "gnsscorr_device_count",
    "gnsscorr_device_pci_bus_id", "gnsscorr_hip_runtime", "gnsscorr_device_lds_bytes",
    "gnsscorr_track_create", "gnsscorr_track_destroy", "gnsscorr_track_max_dumps",
    "gnsscorr_track_set_layout",
    "gnsscorr_pack2", "gnsscorr_track_if_bytes",
    "gnsscorr_track", "gnsscorr_track_dev", "gnsscorr_track_next_tic",
    "gnsscorr_track_replay_dev", "gnsscorr_track_get_state", "gnsscorr_track_set_state",
    "gnsscorr_track_sync", "gnsscorr_track_stream",
    "gnsscorr_acq_create", "gnsscorr_acq_destroy", "gnsscorr_acq_set_codes",
    "gnsscorr_acq_search", "gnsscorr_acq_search_dev", "gnsscorr_acq_power_row",
    "gnsscorr_acq_spectra_dev", "gnsscorr_acq_correlate_dev", "gnsscorr_acq_select_dev",
    "gnsscorr_acq_sync", "gnsscorr_acq_stream", "gnsscorr_acq_set_coherent",
    "gnsscorr_acq_set_records", "gnsscorr_acq_set_group_records", "gnsscorr_acq_set_prn_codes",
    "gnsscorr_sgt_loop_coefs", "gnsscorr_sgt_init_chan", "gnsscorr_sgt_create",
    "gnsscorr_sgt_destroy", "gnsscorr_sgt_track_dev", "gnsscorr_sgt_track", "gnsscorr_sgt_sync",
    "gnsscorr_sgt_stream", "gnsscorr_sgt_replay", "gnsscorr_sgt_replay_dev",
    "gnsscorr_sdr_prn_codes", "gnsscorr_sdr_sine_gen", "gnsscorr_sdr_acq_create",
    "gnsscorr_sdr_acq_destroy", "gnsscorr_sdr_acq_strong", "gnsscorr_sdr_acq_strong_dev",
    "gnsscorr_sdr_channel_start", "gnsscorr_sdr_channel_accum_dev", "gnsscorr_sdr_track_dev",
    "gnsscorr_sdr_acq_sync", "gnsscorr_sdr_acq_stream", "gnsscorr_sdr_acq_prep_dev",
    "gnsscorr_sdr_acq_search_dev", "gnsscorr_sdr_acq_acquire",
    "gnsscorr_sdr_corr_create", "gnsscorr_sdr_corr_destroy", "gnsscorr_sdr_init_chan",
    "gnsscorr_sdr_accum_dev", "gnsscorr_sdr_correlate", "gnsscorr_sdr_corr_sync",
    "gnsscorr_sdr_corr_stream", "gnsscorr_sdr_corr_device",
    "gnsscorr_sdr_gn3s_products", "gnsscorr_sdr_fe_create", "gnsscorr_sdr_fe_destroy",
    "gnsscorr_sdr_gn3s_dev", "gnsscorr_sdr_gn3s", "gnsscorr_sdr_downsample_count",
    "gnsscorr_sdr_downsample_dev", "gnsscorr_sdr_fe_sync", "gnsscorr_sdr_fe_stream",
    "gnsscorr_osg_loop_cfg_init", "gnsscorr_osg_loop_reset", "gnsscorr_osg_isr_dev",
    "gnsscorr_osg_closed_loop_dev",
    "gnsscorr_dev_alloc", "gnsscorr_dev_free", "gnsscorr_memcpy_htod", "gnsscorr_memcpy_dtoh",
    "gnsscorr_dev_synchronize", "gnsscorr_event_create", "gnsscorr_event_record",
    "gnsscorr_stream_wait_event",
    "gnsscorr_event_elapsed_ms", "gnsscorr_event_destroy", "gnsscorr_dev_fill_if2",
    "gnsscorr_ifgen", "gnsscorr_ca_code", "gnsscorr_st_code", "gnsscorr_sample_code",
    "correlator_init", "Sim_GP2021_int", "gnsscorr_osg_configure", "gnsscorr_osg_get_state",
]
EXPORTED_DATA = ["REG_read", "REG_write", "Carrier_DCO_Delta", "Code_DCO_Delta",
                 "gps_code_ref", "gps_carrier_ref", "glonass_code_ref",
                 "glonass_carrier_ref", "d_freq"]

_lib = None


class GnssCorrError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libgnsscorr.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GnssCorrError(f"{LIB_PATH} not built (run `make -C gnss-sdr.ru_amd`)")
    L = C.CDLL(LIB_PATH)  # RTLD_LOCAL: never interpose REG_read etc. into other libraries
    P, I, I64, D, U64 = C.c_void_p, C.c_int, C.c_int64, C.c_double, C.c_uint64
    sig = {
        "gnsscorr_last_error": (C.c_char_p, []),
        "gnsscorr_version": (C.c_char_p, []),
        "gnsscorr_device_count": (I, []),
        "gnsscorr_device_pci_bus_id": (I, [I, P, I]),
        "gnsscorr_device_lds_bytes": (I, [I]),
        "gnsscorr_hip_runtime": (I, [P, I, P]),
        "gnsscorr_track_create": (I, [C.POINTER(P), C.POINTER(TrackCfg)]),
        "gnsscorr_track_destroy": (I, [P]),
        "gnsscorr_track_set_layout": (I, [P, I]),
        "gnsscorr_track_max_dumps": (I, [P]),
        "gnsscorr_track": (I, [P, P, I64, I, I64, P, P, P, C.POINTER(I)]),
        "gnsscorr_track_dev": (I, [P, P, I64, I64, P, P, P, I64]),
        "gnsscorr_track_next_tic": (I64, [P, I64]),
        "gnsscorr_track_if_bytes": (I64, [P, I64]),
        "gnsscorr_pack2": (I, [P, I64, P]),
        "gnsscorr_track_replay_dev": (I, [P, P, I64, I64, I, P, P]),
        "gnsscorr_track_get_state": (I, [P, P]),
        "gnsscorr_track_set_state": (I, [P, P]),
        "gnsscorr_track_sync": (I, [P]),
        "gnsscorr_track_stream": (P, [P]),
        "gnsscorr_acq_create": (I, [C.POINTER(P), C.POINTER(AcqCfg)]),
        "gnsscorr_acq_destroy": (I, [P]),
        "gnsscorr_acq_set_codes": (I, [P, I, P]),
        "gnsscorr_acq_search": (I, [P, P, I, I, I, I, P, I, I, P, P, I, P, P]),
        "gnsscorr_acq_search_dev": (I, [P, P, I, I, I, I, P, I, I, P, P, I, P, P]),
        "gnsscorr_acq_power_row": (I, [P, P, I, I, I, D, I, P]),
        "gnsscorr_acq_spectra_dev": (I, [P, P, I, I, I, P]),
        "gnsscorr_acq_correlate_dev": (I, [P, I, I, P, I, I, P, P, I, P, P]),
        "gnsscorr_acq_select_dev": (I, [P, I, I, P, P, P, P]),
        "gnsscorr_acq_sync": (I, [P]),
        "gnsscorr_acq_set_coherent": (I, [P, I]),
        "gnsscorr_acq_set_records": (I, [P, I]),
        "gnsscorr_acq_set_group_records": (I, [P, P]),
        "gnsscorr_acq_set_prn_codes": (I, [P, I, P]),
        "gnsscorr_acq_stream": (P, [P]),
        "gnsscorr_sgt_loop_coefs": (None, [C.POINTER(SgtCfg)] + [C.POINTER(D)] * 5),
        "gnsscorr_sgt_init_chan": (I, [C.POINTER(SgtCfg), I, I, I64, I64, D, P]),
        "gnsscorr_sgt_create": (I, [C.POINTER(P), C.POINTER(SgtCfg)]),
        "gnsscorr_sgt_destroy": (I, [P]),
        "gnsscorr_sgt_track_dev": (I, [P, P, I64, I64, I, P, I, I, P]),
        "gnsscorr_sgt_track": (I, [P, P, I64, I64, I, P, I, I, P]),
        "gnsscorr_sgt_replay": (I, [P, I, P, I, P, P]),
        "gnsscorr_sgt_replay_dev": (I, [P, I, P, I, P, P]),
        "gnsscorr_sgt_sync": (I, [P]),
        "gnsscorr_sgt_stream": (P, [P]),
        "gnsscorr_sdr_prn_codes": (I, [P]),
        "gnsscorr_sdr_sine_gen": (None, [P, D, D, I]),
        "gnsscorr_sdr_acq_create": (I, [C.POINTER(P), C.POINTER(SdrAcqCfg)]),
        "gnsscorr_sdr_acq_destroy": (I, [P]),
        "gnsscorr_sdr_acq_strong": (I, [P, P, I, I, P, I, I, P]),
        "gnsscorr_sdr_acq_strong_dev": (I, [P, P, I, I, P, I, I, P]),
        "gnsscorr_sdr_acq_sync": (I, [P]),
        "gnsscorr_sdr_acq_prep_dev": (I, [P, I, P, I]),
        "gnsscorr_sdr_channel_start": (I, [P, I, I, I, I]),
        "gnsscorr_sdr_channel_accum_dev": (I, [P, I, I, P, P, P, P, P, I, P]),
        "gnsscorr_sdr_track_dev": (I, [P, P, I, I, I, P, P, P, P, P, P, I, P, P, P, I, P]),
        "gnsscorr_sdr_acq_search_dev": (I, [P, I, I, I, P, I, I, P]),
        "gnsscorr_sdr_acq_acquire": (I, [P, I, P, I, I, P, I, I, P]),
        "gnsscorr_sdr_acq_stream": (P, [P]),
        "gnsscorr_sdr_corr_create": (I, [C.POINTER(P), C.POINTER(SdrCorrCfg)]),
        "gnsscorr_sdr_corr_destroy": (I, [P]),
        "gnsscorr_sdr_init_chan": (I, [P, I, I, I, D]),
        "gnsscorr_sdr_accum_dev": (I, [P, P, I, P, P]),
        "gnsscorr_sdr_correlate": (I, [P, P, I, I, P, P, P, P, P]),
        "gnsscorr_sdr_corr_sync": (I, [P]),
        "gnsscorr_sdr_corr_stream": (P, [P]),
        "gnsscorr_sdr_corr_device": (I, [P]),
        "gnsscorr_sdr_gn3s_products": (None, [P]),
        "gnsscorr_osg_loop_cfg_init": (None, [P, D, D, D, I, I, D, C.c_long, C.c_long, C.c_long,
                                              C.c_long, C.c_long, I]),
        "gnsscorr_osg_loop_reset": (None, [P, I, P, P, P]),
        "gnsscorr_osg_isr_dev": (I, [P, P, I, P, P, P]),
        "gnsscorr_osg_closed_loop_dev": (I, [P, P, P, I64, I64, I, I, P, P, P, P]),
        "gnsscorr_sdr_fe_create": (I, [C.POINTER(P), I]),
        "gnsscorr_sdr_fe_destroy": (I, [P]),
        "gnsscorr_sdr_gn3s_dev": (I, [P, P, I, I, C.POINTER(C.c_uint32), C.c_uint32, P]),
        "gnsscorr_sdr_gn3s": (I, [P, P, I, I, C.POINTER(C.c_uint32), C.c_uint32, P]),
        "gnsscorr_sdr_downsample_count": (I, [I, D, D, P]),
        "gnsscorr_sdr_downsample_dev": (I, [P, P, I, D, D, P, C.POINTER(C.c_int)]),
        "gnsscorr_sdr_fe_sync": (I, [P]),
        "gnsscorr_sdr_fe_stream": (P, [P]),
        "gnsscorr_dev_alloc": (I, [I, C.c_size_t, C.POINTER(P)]),
        "gnsscorr_dev_free": (I, [I, P]),
        "gnsscorr_memcpy_htod": (I, [I, P, P, C.c_size_t]),
        "gnsscorr_memcpy_dtoh": (I, [I, P, P, C.c_size_t]),
        "gnsscorr_dev_synchronize": (I, [I]),
        "gnsscorr_event_create": (I, [I, C.POINTER(P)]),
        "gnsscorr_event_record": (I, [P, P]),
        "gnsscorr_stream_wait_event": (I, [P, P]),
        "gnsscorr_event_elapsed_ms": (I, [P, P, C.POINTER(C.c_float)]),
        "gnsscorr_event_destroy": (I, [P]),
        "gnsscorr_dev_fill_if2": (I, [I, P, C.c_size_t, U64]),
        "gnsscorr_ifgen": (I, [P, I64, I, D, D, D, I, P, U64]),
        "gnsscorr_ca_code": (I, [I, P]),
        "gnsscorr_st_code": (I, [P]),
        "gnsscorr_sample_code": (I, [P, I, D, D, I, P]),
        "correlator_init": (None, [D]),
        "Sim_GP2021_int": (None, [P, C.c_long]),
        "gnsscorr_osg_configure": (I, [D, D, D, D, I, I, I, I, D, I]),
        "gnsscorr_osg_get_state": (I, [P]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):
            continue  # reported by tests/test_abi.py
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().gnsscorr_last_error().decode(errors="replace")
        raise GnssCorrError(f"{what} failed ({rc}): {msg}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _if_bytes(a) -> np.ndarray:
    """IF samples as the C ABI's int8 byte buffer (packed data may come as uint8)."""
    a = np.ascontiguousarray(a)
    return a.view(np.int8) if a.dtype == np.uint8 else np.ascontiguousarray(a, np.int8)


def iq_flags(iq, packed=False) -> int:
    """The `iq` argument of the C ABI: GNSSCORR_IF_* flags (iq may already be flags)."""
    f = int(iq)
    return f | IF_PACKED2 if packed else f


def pack2(levels) -> np.ndarray:
    """int8 levels in {-3,-1,1,3} -> GNSSCORR_IF_PACKED2 bytes (gnsscorr_pack2)."""
    lv = np.ascontiguousarray(levels, np.int8).ravel()
    out = np.empty((lv.size + 3) // 4, np.uint8)
    _check(lib().gnsscorr_pack2(_ptr(lv), lv.size, _ptr(out)), "gnsscorr_pack2")
    return out


def device_count() -> int:
    return int(lib().gnsscorr_device_count())


def device_lds_bytes(device: int = 0) -> int:
    """LDS bytes a workgroup may allocate on the device (gnsscorr_device_lds_bytes)."""
    return int(lib().gnsscorr_device_lds_bytes(device))


def pci_bus_id(device: int = 0) -> str:
    buf = C.create_string_buffer(64)
    _check(lib().gnsscorr_device_pci_bus_id(device, buf, 64), "gnsscorr_device_pci_bus_id")
    return buf.value.decode()


def hip_runtime() -> dict:
    """The libamdhip64 libgnsscorr's HIP calls bind to (gnsscorr_hip_runtime), its
    hipRuntimeGetVersion, and every libamdhip64 the process has mapped."""
    buf = C.create_string_buffer(4096)
    ver = C.c_int(0)
    _check(lib().gnsscorr_hip_runtime(buf, 4096, C.byref(ver)), "gnsscorr_hip_runtime")
    mapped = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line and line.split()[-1] not in mapped:
                    mapped.append(line.split()[-1])
    except OSError:
        pass
    return dict(bound=os.path.realpath(buf.value.decode()), version=ver.value, mapped=mapped)


# ---------------------------------------------------------------- device memory
class DevBuf:
    """A HIP device allocation owned by libgnsscorr (no other GPU runtime)."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device = device
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _check(lib().gnsscorr_dev_alloc(device, self.nbytes, C.byref(p)), "gnsscorr_dev_alloc")
        self.ptr = p.value

    @classmethod
    def from_array(cls, a: np.ndarray, device: int = 0) -> "DevBuf":
        a = np.ascontiguousarray(a)
        b = cls(max(a.nbytes, 1), device)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        _check(lib().gnsscorr_memcpy_htod(self.device, self.ptr + offset, _ptr(a), a.nbytes),
               "gnsscorr_memcpy_htod")

    def download(self, dtype, count: int = -1, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        if count < 0:
            count = (self.nbytes - offset) // dt.itemsize
        out = np.empty(count, dt)
        _check(lib().gnsscorr_memcpy_dtoh(self.device, _ptr(out), self.ptr + offset, out.nbytes),
               "gnsscorr_memcpy_dtoh")
        return out

    def fill_if2(self, seed: int):
        _check(lib().gnsscorr_dev_fill_if2(self.device, self.ptr, self.nbytes, seed),
               "gnsscorr_dev_fill_if2")

    def free(self):
        if getattr(self, "ptr", None):
            lib().gnsscorr_dev_free(self.device, self.ptr)
            self.ptr = None

    __del__ = free


def dev_synchronize(device: int = 0):
    _check(lib().gnsscorr_dev_synchronize(device), "gnsscorr_dev_synchronize")


class Event:
    """hipEvent_t wrapper for timing on a specific HIP stream."""

    def __init__(self, device: int = 0):
        p = C.c_void_p()
        _check(lib().gnsscorr_event_create(device, C.byref(p)), "gnsscorr_event_create")
        self.h = p

    def record(self, stream: int):
        _check(lib().gnsscorr_event_record(self.h, stream), "gnsscorr_event_record")

    def wait_on(self, stream: int):
        """Work queued on `stream` from now on waits for this event."""
        _check(lib().gnsscorr_stream_wait_event(stream, self.h), "gnsscorr_stream_wait_event")

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float()
        _check(lib().gnsscorr_event_elapsed_ms(self.h, end.h, C.byref(ms)),
               "gnsscorr_event_elapsed_ms")
        return float(ms.value)

    def __del__(self):
        if getattr(self, "h", None):
            lib().gnsscorr_event_destroy(self.h)
            self.h = None


# ---------------------------------------------------------------- host utils
def ca_code(prn: int) -> np.ndarray:
    out = np.empty(1023, np.int8)
    _check(lib().gnsscorr_ca_code(prn, _ptr(out)), "gnsscorr_ca_code")
    return out


def st_code() -> np.ndarray:
    out = np.empty(511, np.int8)
    _check(lib().gnsscorr_st_code(_ptr(out)), "gnsscorr_st_code")
    return out


def sample_code(chips: np.ndarray, code_rate: float, fs: float, n: int) -> np.ndarray:
    chips = np.ascontiguousarray(chips, np.int8)
    out = np.empty(n, np.int8)
    _check(lib().gnsscorr_sample_code(_ptr(chips), len(chips), code_rate, fs, n, _ptr(out)),
           "gnsscorr_sample_code")
    return out


def make_sigs(sigs) -> np.ndarray:
    """sigs: list of dicts with keys of SIG (missing keys default to 0)."""
    a = np.zeros(len(sigs), SIG)
    for i, s in enumerate(sigs):
        for k, v in s.items():
            a[i][k] = v
    return a


def ifgen(nsamp: int, sigs=(), fs=16.368e6, if_gps=2.42e6, if_glo=1.0e6, iq=True,
          seed=0x5EED0000) -> np.ndarray:
    """Deterministic synthetic 2-bit IF as int8 (interleaved I,Q when iq)."""
    sa = make_sigs(sigs) if not isinstance(sigs, np.ndarray) else sigs
    out = np.empty(nsamp * (2 if iq else 1), np.int8)
    _check(lib().gnsscorr_ifgen(_ptr(out), nsamp, int(iq), fs, if_gps, if_glo, len(sa),
                                _ptr(sa) if len(sa) else None, seed), "gnsscorr_ifgen")
    return out


# ---------------------------------------------------------------- tracking
class TrackCtx:
    """Batched GP2021-semantics tracking correlator context (one per GPU)."""

    def __init__(self, n_channels: int, iq: bool = True, device: int = 0,
                 max_nsamp: int = 65536, samp_rate: float = 16.368e6,
                 tic_period: float = 0.0, packed: bool = False):
        self.n_channels = n_channels
        self.iq = bool(int(iq) & IF_IQ)
        self.packed = bool(packed or int(iq) & IF_PACKED2)
        cfg = TrackCfg(n_channels, iq_flags(self.iq, self.packed), device, max_nsamp, samp_rate,
                       tic_period)
        h = C.c_void_p()
        _check(lib().gnsscorr_track_create(C.byref(h), C.byref(cfg)), "gnsscorr_track_create")
        self.h = h
        self.max_dumps = lib().gnsscorr_track_max_dumps(h)

    def set_layout(self, one_stream_per_channel: bool):
        """gnsscorr_track_set_layout: per-channel LDS staging of int8 C_s = 1 streams."""
        _check(lib().gnsscorr_track_set_layout(self.h, int(bool(one_stream_per_channel))),
               "gnsscorr_track_set_layout")

    def close(self):
        if getattr(self, "h", None):
            lib().gnsscorr_track_destroy(self.h)
            self.h = None

    __del__ = close

    def track(self, if_samples: np.ndarray, nsamp: int, cmds: np.ndarray, n_streams: int = 1,
              stream_stride: int = 0, all_dumps: bool = False):
        if_samples = _if_bytes(if_samples)
        cmds = np.ascontiguousarray(cmds, NCO_CMD)
        assert len(cmds) == self.n_channels
        res = np.zeros(self.n_channels, TRACK_RESULT)
        dumps = np.zeros((self.n_channels, self.max_dumps, 6), np.int32) if all_dumps else None
        tic = C.c_int(0)
        _check(lib().gnsscorr_track(self.h, _ptr(if_samples), stream_stride, n_streams, nsamp,
                                    _ptr(cmds), _ptr(res),
                                    _ptr(dumps) if dumps is not None else None, C.byref(tic)),
               "gnsscorr_track")
        return (res, bool(tic.value), dumps) if all_dumps else (res, bool(tic.value))

    def track_dev(self, d_if: int, stream_stride: int, nsamp: int, d_cmds: int, d_res: int,
                  d_dumps: int = 0, tic_count: int = -1):
        _check(lib().gnsscorr_track_dev(self.h, d_if, stream_stride, nsamp, d_cmds, d_res,
                                        d_dumps or None, tic_count), "gnsscorr_track_dev")

    def replay_dev(self, d_if: int, stream_stride: int, nsamp: int, n_steps: int, d_cmds: int,
                   d_res: int):
        _check(lib().gnsscorr_track_replay_dev(self.h, d_if, stream_stride, nsamp, n_steps,
                                               d_cmds, d_res), "gnsscorr_track_replay_dev")

    def if_bytes(self, samples: int) -> int:
        """Bytes of `samples` samples of one stream in this context's format."""
        return int(lib().gnsscorr_track_if_bytes(self.h, samples))

    def next_tic(self, nsamp: int) -> int:
        return int(lib().gnsscorr_track_next_tic(self.h, nsamp))

    def get_state(self) -> np.ndarray:
        st = np.zeros(self.n_channels, CHAN_STATE)
        _check(lib().gnsscorr_track_get_state(self.h, _ptr(st)), "gnsscorr_track_get_state")
        return st

    def set_state(self, st: np.ndarray):
        st = np.ascontiguousarray(st, CHAN_STATE)
        _check(lib().gnsscorr_track_set_state(self.h, _ptr(st)), "gnsscorr_track_set_state")

    def sync(self):
        _check(lib().gnsscorr_track_sync(self.h), "gnsscorr_track_sync")

    @property
    def stream(self) -> int:
        return lib().gnsscorr_track_stream(self.h)


# ---------------------------------------------------------------- acquisition
class AcqCtx:
    """Parallel code-phase acquisition context (SoftGNSS acquisition.sci semantics)."""

    def __init__(self, samp_rate: float = 16.368e6, n_samples: int = 16368, device: int = 0,
                 max_freqs: int = 1024, max_blocks: int = 16, max_codes: int = 64,
                 precision: int = ACQ_F64):
        cfg = AcqCfg(samp_rate, n_samples, device, max_freqs, max_blocks, max_codes, precision)
        self.precision = precision
        h = C.c_void_p()
        _check(lib().gnsscorr_acq_create(C.byref(h), C.byref(cfg)), "gnsscorr_acq_create")
        self.h = h
        self.n = n_samples
        self.fs = samp_rate
        self.records = 1

    def close(self):
        if getattr(self, "h", None):
            lib().gnsscorr_acq_destroy(self.h)
            self.h = None

    __del__ = close

    def set_codes(self, codes: np.ndarray):
        codes = np.ascontiguousarray(codes, np.int8).reshape(-1, self.n)
        _check(lib().gnsscorr_acq_set_codes(self.h, codes.shape[0], _ptr(codes)),
               "gnsscorr_acq_set_codes")

    def set_prn_codes(self, code_ids):
        """gnsscorr_acq_set_prn_codes: replicas generated on the device from code ids
        (1..32: GPS C/A PRN; CODE_GLO_ST: the GLONASS ST code), then their spectra
        (acquisition.sci:91-95).  Asynchronous on the context stream."""
        ids = np.ascontiguousarray(code_ids, np.int32)
        _check(lib().gnsscorr_acq_set_prn_codes(self.h, len(ids), _ptr(ids)),
               "gnsscorr_acq_set_prn_codes")

    def search(self, if_samples, n_blocks, freqs, group_code, group_freq, spc=16, iq=True,
               mode=ACQ_BEST_OF_BLOCKS):
        if_samples = _if_bytes(if_samples)
        freqs = np.ascontiguousarray(freqs, np.float64)
        group_code = np.ascontiguousarray(group_code, np.int32)
        group_freq = np.ascontiguousarray(group_freq, np.int32).reshape(len(group_code), -1)
        G, B = group_freq.shape
        R = 1 if getattr(self, "_group_rec", None) is not None else self.records
        rows = np.zeros(R * G * B, ACQ_ROW)
        res = np.zeros(R * G, ACQ_RESULT)
        _check(lib().gnsscorr_acq_search(self.h, _ptr(if_samples), int(iq), n_blocks, mode,
                                         len(freqs), _ptr(freqs), G, B, _ptr(group_code),
                                         _ptr(group_freq), spc, _ptr(rows), _ptr(res)),
               "gnsscorr_acq_search")
        if R == 1:
            return res, rows.reshape(G, B)
        return res.reshape(R, G), rows.reshape(R, G, B)

    def set_records(self, n_records: int):
        """Records per search (fp64): n_records IF records end to end, searched
        in one launch; search() then returns (R, G) results and (R, G, B) rows."""
        _check(lib().gnsscorr_acq_set_records(self.h, int(n_records)), "gnsscorr_acq_set_records")
        if int(n_records) != getattr(self, "records", 1):
            self._group_rec = None   # the library drops a per-group table on a count change
        self.records = int(n_records)

    def set_group_records(self, d_group_rec):
        """Per-group IF records (gnsscorr_acq_set_group_records): a device int32 array
        (DevBuf or pointer), group g searched on record d_group_rec[g] only; None: off."""
        ptr = None if d_group_rec is None else getattr(d_group_rec, "ptr", d_group_rec)
        _check(lib().gnsscorr_acq_set_group_records(self.h, ptr),
               "gnsscorr_acq_set_group_records")
        self._group_rec = d_group_rec   # keep the device array alive

    def set_coherent(self, coh_ms: int):
        """settings.acqCohIntegration: code periods per coherent block (default 1)."""
        _check(lib().gnsscorr_acq_set_coherent(self.h, int(coh_ms)), "gnsscorr_acq_set_coherent")

    def search_dev(self, d_if, n_blocks, n_freqs, d_freqs, n_groups, n_bins, d_group_code,
                   d_group_freq, d_rows, d_res, spc=16, iq=True, mode=ACQ_BEST_OF_BLOCKS):
        _check(lib().gnsscorr_acq_search_dev(self.h, d_if, int(iq), n_blocks, mode, n_freqs,
                                             d_freqs, n_groups, n_bins, d_group_code,
                                             d_group_freq, spc, d_rows, d_res),
               "gnsscorr_acq_search_dev")

    def spectra_dev(self, d_if, n_blocks, n_freqs, d_freqs, iq=True):
        _check(lib().gnsscorr_acq_spectra_dev(self.h, d_if, int(iq), n_blocks, n_freqs, d_freqs),
               "gnsscorr_acq_spectra_dev")

    def correlate_dev(self, n_blocks, d_freqs, n_groups, n_bins, d_group_code, d_group_freq,
                      d_rows=None, d_res=None, spc=16, mode=ACQ_BEST_OF_BLOCKS):
        _check(lib().gnsscorr_acq_correlate_dev(self.h, n_blocks, mode, d_freqs, n_groups, n_bins,
                                                d_group_code, d_group_freq, spc, d_rows or None,
                                                d_res or None), "gnsscorr_acq_correlate_dev")

    def select_dev(self, n_groups, n_bins, d_freqs, d_group_freq, d_rows, d_res):
        _check(lib().gnsscorr_acq_select_dev(self.h, n_groups, n_bins, d_freqs, d_group_freq,
                                             d_rows, d_res), "gnsscorr_acq_select_dev")

    def power_row(self, if_samples, n_blocks, block, freq, code, iq=True) -> np.ndarray:
        if_samples = _if_bytes(if_samples)
        out = np.empty(self.n, np.float64)
        _check(lib().gnsscorr_acq_power_row(self.h, _ptr(if_samples), int(iq), n_blocks, block,
                                            freq, code, _ptr(out)), "gnsscorr_acq_power_row")
        return out

    def sync(self):
        _check(lib().gnsscorr_acq_sync(self.h), "gnsscorr_acq_sync")

    @property
    def stream(self) -> int:
        return lib().gnsscorr_acq_stream(self.h)


# ---------------------------------------------------------------- SoftGNSS float tracking
def sgt_cfg(system: int, device: int = 0, **kw) -> SgtCfg:
    """initSettings.sci defaults (GLONASS/L1:41-107, GPS/L1:41-95); keyword overrides
    use the Scilab names (samplingFreq, IF, dllCorrelatorSpacing, fileType, ...)."""
    glo = system == 1
    d = dict(samplingFreq=16e6, codeFreqBasis=0.511e6 if glo else 1.023e6,
             codeLength=511 if glo else 1023, IF=1e6 if glo else 2.42e6,
             L1_IF_step=0.5625e6 if glo else 0.0, GLONASS_zero_channel=1602e6 if glo else 0.0,
             dllCorrelatorSpacing=0.05 if glo else 0.2, dllNoiseBandwidth=0.5 if glo else 0.1,
             dllDampingRatio=0.7, pllNoiseBandwidth=25.0, fllNoiseBandwidth=250.0, fileType=2,
             switchIQ=0, codeNcoVariant=0, absSampleVariant=0)
    unknown = set(kw) - set(d) - {"system"}
    if unknown:
        raise ValueError(f"unknown settings {sorted(unknown)}")
    d.update(kw)
    return SgtCfg(system, d["fileType"], d["switchIQ"], d["codeLength"], device, 0,
                  d["samplingFreq"], d["codeFreqBasis"], d["IF"], d["L1_IF_step"],
                  d["GLONASS_zero_channel"], d["dllCorrelatorSpacing"], d["dllNoiseBandwidth"],
                  d["dllDampingRatio"], d["pllNoiseBandwidth"], d["fllNoiseBandwidth"],
                  d["codeNcoVariant"], d["absSampleVariant"])


class SgtCtx:
    """SoftGNSS float tracking (tracking.sci) for many channels over HBM-resident records."""

    def __init__(self, system: int, device: int = 0, **settings):
        self.cfg = sgt_cfg(system, device, **settings)
        h = C.c_void_p()
        _check(lib().gnsscorr_sgt_create(C.byref(h), C.byref(self.cfg)), "gnsscorr_sgt_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().gnsscorr_sgt_destroy(self.h)
            self.h = None

    __del__ = close

    def loop_coefs(self):
        v = [C.c_double() for _ in range(5)]
        lib().gnsscorr_sgt_loop_coefs(C.byref(self.cfg), *[C.byref(x) for x in v])
        return tuple(x.value for x in v)     # tau1code, tau2code, k1, k2, k3

    def init_chans(self, code_ids, code_phases_1b, acq_freqs, streams=None, skip=0):
        n = len(code_ids)
        out = np.zeros(n, SGT_CHAN)
        streams = np.zeros(n, np.int64) if streams is None else np.asarray(streams)
        for i in range(n):
            _check(lib().gnsscorr_sgt_init_chan(C.byref(self.cfg), int(code_ids[i]),
                                                int(streams[i]), int(skip),
                                                int(code_phases_1b[i]), float(acq_freqs[i]),
                                                out[i:i + 1].ctypes.data),
                   "gnsscorr_sgt_init_chan")
        return out

    def track(self, d_if, stride, n_samples, chans, n_epochs, closed_loop=True):
        """Host channel array in/out; returns epochs [n_ch, n_epochs]."""
        assert chans.dtype == SGT_CHAN and chans.flags.c_contiguous
        ep = np.zeros((len(chans), n_epochs), SGT_EPOCH)
        _check(lib().gnsscorr_sgt_track(self.h, d_if, stride, n_samples, len(chans),
                                        _ptr(chans), n_epochs, int(closed_loop), _ptr(ep)),
               "gnsscorr_sgt_track")
        return ep

    def track_dev(self, d_if, stride, n_samples, n_ch, d_chan, n_epochs, d_epochs,
                  closed_loop=True):
        _check(lib().gnsscorr_sgt_track_dev(self.h, d_if, stride, n_samples, n_ch, d_chan,
                                            n_epochs, int(closed_loop), d_epochs),
               "gnsscorr_sgt_track_dev")

    def replay(self, chans, sums):
        """The loop half on given sums [n_ch, n_epochs, 6] (I_E, I_P, I_L, Q_E, Q_P,
        Q_L); host channel array in/out; returns epochs [n_ch, n_epochs]."""
        assert chans.dtype == SGT_CHAN and chans.flags.c_contiguous
        sums = np.ascontiguousarray(sums, dtype=np.float64)
        n_ch, n_ep = sums.shape[0], sums.shape[1]
        assert sums.shape == (len(chans), n_ep, 6)
        ep = np.zeros((n_ch, n_ep), SGT_EPOCH)
        _check(lib().gnsscorr_sgt_replay(self.h, n_ch, _ptr(chans), n_ep, _ptr(sums), _ptr(ep)),
               "gnsscorr_sgt_replay")
        return ep

    def sync(self):
        _check(lib().gnsscorr_sgt_sync(self.h), "gnsscorr_sgt_sync")

    @property
    def stream(self) -> int:
        return lib().gnsscorr_sgt_stream(self.h)


# ---------------------------------------------------------------- GPS-SDR integer acquisition
def sdr_prn_codes() -> np.ndarray:
    """PRN_Codes (51, 2048, 2) int16 as gen_fft_codes.m builds them."""
    out = np.zeros((51, 2048, 2), np.int16)
    _check(lib().gnsscorr_sdr_prn_codes(_ptr(out)), "gnsscorr_sdr_prn_codes")
    return out


def sdr_sine_gen(f: float, n: int = 2048, fs: float = 2048000.0) -> np.ndarray:
    out = np.zeros((n, 2), np.int16)
    lib().gnsscorr_sdr_sine_gen(_ptr(out), f, fs, n)
    return out


class SdrAcqCtx:
    """GPS-SDR strong (1 ms, int16 FFT) acquisition, bit-exact with the reference."""

    def __init__(self, fif: float = 38400.0, device: int = 0, saturate: bool = False):
        h = C.c_void_p()
        _check(lib().gnsscorr_sdr_acq_create(C.byref(h), C.byref(SdrAcqCfg(fif, device,
                                                                             int(saturate)))),
               "gnsscorr_sdr_acq_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().gnsscorr_sdr_acq_destroy(self.h)
            self.h = None

    __del__ = close

    def strong(self, buffers, svs, doppmin=-15000, doppmax=15000) -> np.ndarray:
        """buffers: (n_rec, 2048, 2) or (2048, 2) int16; returns SDR_RESULT [n_rec, n_sv]."""
        b = np.ascontiguousarray(buffers, np.int16).reshape(-1, 2048, 2)
        svs = np.ascontiguousarray(svs, np.int32)
        res = np.zeros((b.shape[0], len(svs)), SDR_RESULT)
        _check(lib().gnsscorr_sdr_acq_strong(self.h, _ptr(b), b.shape[0], len(svs), _ptr(svs),
                                             doppmin, doppmax, _ptr(res)),
               "gnsscorr_sdr_acq_strong")
        return res

    def acquire(self, acq_type, buffers, svs, doppmin=-15000, doppmax=15000) -> np.ndarray:
        """Acquisition::Acquire for one request type (doPrepIF + doAcqStrong /
        doAcqMedium / doAcqWeak).  buffers: (n_rec, ms*2048, 2) int16 with ms =
        1 / 10 / 310; returns SDR_RESULT [n_rec, n_sv].  Medium and weak preps
        update the context's persistent per-record row store."""
        ms = SDR_ACQ_MS[acq_type]
        b = np.ascontiguousarray(buffers, np.int16).reshape(-1, ms * 2048, 2)
        svs = np.ascontiguousarray(svs, np.int32)
        res = np.zeros((b.shape[0], len(svs)), SDR_RESULT)
        _check(lib().gnsscorr_sdr_acq_acquire(self.h, acq_type, _ptr(b), b.shape[0], len(svs),
                                              _ptr(svs), doppmin, doppmax, _ptr(res)),
               "gnsscorr_sdr_acq_acquire")
        return res

    def prep_dev(self, acq_type, d_buff, n_rec):
        _check(lib().gnsscorr_sdr_acq_prep_dev(self.h, acq_type, d_buff, n_rec),
               "gnsscorr_sdr_acq_prep_dev")

    def search_dev(self, acq_type, n_rec, n_sv, d_svs, d_res, doppmin=-15000, doppmax=15000):
        _check(lib().gnsscorr_sdr_acq_search_dev(self.h, acq_type, n_rec, n_sv, d_svs, doppmin,
                                                 doppmax, d_res), "gnsscorr_sdr_acq_search_dev")

    def strong_dev(self, d_buff, n_rec, n_sv, d_svs, d_res, doppmin=-15000, doppmax=15000):
        _check(lib().gnsscorr_sdr_acq_strong_dev(self.h, d_buff, n_rec, n_sv, d_svs, doppmin,
                                                 doppmax, d_res), "gnsscorr_sdr_acq_strong_dev")

    def sync(self):
        _check(lib().gnsscorr_sdr_acq_sync(self.h), "gnsscorr_sdr_acq_sync")

    @property
    def stream(self) -> int:
        return lib().gnsscorr_sdr_acq_stream(self.h)


class OsgLoopCfg(C.Structure):
    _fields_ = [("carrier_ref", C.c_int64), ("code_ref", C.c_int64), ("d_freq", C.c_int64),
                ("fll_i1", C.c_int32), ("fll_i2", C.c_int32), ("fll_i3", C.c_int32),
                ("dll_i1", C.c_int32), ("dll_i2", C.c_int32), ("acq_thresh", C.c_int32),
                ("confirm_m", C.c_int32), ("n_of_m_thresh", C.c_int32),
                ("carrier_shift", C.c_int32), ("code_shift", C.c_int32),
                ("clock_mult", C.c_double)]


def osg_loop_cfg(samp_rate=16.0e6, gps_if=2.42e6, clock_mult=5.0, carrier_bits=30, code_bits=29,
                 bin_width=1000.0, bnp=25, bnf=1400, bnd=2, fll_t_ms=1, dll_t_ms=1,
                 acq_thresh=1800) -> OsgLoopCfg:
    """Receiver loop constants as the reference derives them (globals.h defaults)."""
    cfg = OsgLoopCfg()
    lib().gnsscorr_osg_loop_cfg_init(C.byref(cfg), samp_rate, gps_if, clock_mult, carrier_bits,
                                     code_bits, bin_width, bnp, bnf, bnd, fll_t_ms, dll_t_ms,
                                     acq_thresh)
    return cfg


def osg_loop_reset(cfg: OsgLoopCfg, prns):
    """Start state of every channel (reset_all_correlator_channles) -> (loops, cmds)."""
    prns = np.ascontiguousarray(prns, np.int32)
    loops = np.zeros(len(prns), OSG_LOOP)
    cmds = np.zeros(len(prns), NCO_CMD)
    lib().gnsscorr_osg_loop_reset(C.byref(cfg), len(prns), _ptr(prns), _ptr(loops), _ptr(cmds))
    return loops, cmds


def osg_isr_dev(track: "TrackCtx", cfg: OsgLoopCfg, n_ch, d_loops, d_cmds, d_res):
    _check(lib().gnsscorr_osg_isr_dev(track.h, C.byref(cfg), n_ch, d_loops, d_cmds, d_res),
           "gnsscorr_osg_isr_dev")


def osg_closed_loop_dev(track: "TrackCtx", cfg: OsgLoopCfg, d_if, stream_stride, nsamp, n_calls,
                        n_ch, d_loops, d_cmds, d_res_hist, d_loop_hist=None):
    _check(lib().gnsscorr_osg_closed_loop_dev(track.h, C.byref(cfg), d_if, stream_stride, nsamp,
                                              n_calls, n_ch, d_loops, d_cmds, d_res_hist,
                                              d_loop_hist), "gnsscorr_osg_closed_loop_dev")


GN3S_BLOCK_IN, GN3S_BLOCK_OUT, GN3S_STEP = 20000, 10240, 2557223528


def gn3s_products() -> np.ndarray:
    """The GN3S front end's int16 product table [4 codes, 1024 phases, 2]."""
    out = np.zeros((4, 1024, 2), np.int16)
    lib().gnsscorr_sdr_gn3s_products(_ptr(out))
    return out


def pack_2bit(samples) -> np.ndarray:
    """One-sample-per-byte 2-bit codes -> packed bytes (sample j in bits 2j..2j+1)."""
    s = np.ascontiguousarray(samples, np.uint8).reshape(-1, 4) & 3
    return (s[:, 0] | (s[:, 1] << 2) | (s[:, 2] << 4) | (s[:, 3] << 6)).astype(np.uint8)


class SdrFeCtx:
    """GPS-SDR sample front end: GN3S 2-bit unpack + NCO mix + resample, downsample."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        _check(lib().gnsscorr_sdr_fe_create(C.byref(h), device), "gnsscorr_sdr_fe_create")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            lib().gnsscorr_sdr_fe_destroy(self.h)
            self.h = None

    __del__ = close

    def gn3s(self, data, packed=False, phase=0, step=GN3S_STEP):
        """data: n_blocks * 20000 bytes (or / 4 when packed); returns (CPX [n*10240, 2], phase)."""
        d = np.ascontiguousarray(data, np.uint8).ravel()
        per = GN3S_BLOCK_IN // 4 if packed else GN3S_BLOCK_IN
        nb = d.size // per
        out = np.zeros((nb * GN3S_BLOCK_OUT, 2), np.int16)
        ph = C.c_uint32(phase)
        _check(lib().gnsscorr_sdr_gn3s(self.h, _ptr(d), int(packed), nb, C.byref(ph),
                                       C.c_uint32(step), _ptr(out)), "gnsscorr_sdr_gn3s")
        return out, ph.value

    def gn3s_dev(self, d_in, packed, n_blocks, phase, d_out, step=GN3S_STEP) -> int:
        ph = C.c_uint32(phase)
        _check(lib().gnsscorr_sdr_gn3s_dev(self.h, d_in, int(packed), n_blocks, C.byref(ph),
                                           C.c_uint32(step), d_out), "gnsscorr_sdr_gn3s_dev")
        return ph.value

    def downsample_dev(self, d_src, n_src, fdest, fsource, d_dest) -> int:
        n = C.c_int()
        _check(lib().gnsscorr_sdr_downsample_dev(self.h, d_src, n_src, C.c_double(fdest),
                                                 C.c_double(fsource), d_dest, C.byref(n)),
               "gnsscorr_sdr_downsample_dev")
        return n.value

    @staticmethod
    def downsample_count(n_src, fdest, fsource) -> int:
        return lib().gnsscorr_sdr_downsample_count(n_src, C.c_double(fdest), C.c_double(fsource),
                                                   None)

    def sync(self):
        _check(lib().gnsscorr_sdr_fe_sync(self.h), "gnsscorr_sdr_fe_sync")

    @property
    def stream(self) -> int:
        return lib().gnsscorr_sdr_fe_stream(self.h)


class SdrCorrCtx:
    """GPS-SDR tracking correlator (Correlator class): batched Accum on the GPU,
    Correlate schedule + UpdateState/DumpAccum on the host, channel loop by callback."""

    def __init__(self, device: int = 0, saturate: bool = False):
        h = C.c_void_p()
        _check(lib().gnsscorr_sdr_corr_create(C.byref(h), C.byref(SdrCorrCfg(device,
                                                                               int(saturate)))),
               "gnsscorr_sdr_corr_create")
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().gnsscorr_sdr_corr_destroy(self.h)
            self.h = None

    __del__ = close

    @staticmethod
    def init_chan(sv, acq_code_phase, acq_doppler, packets_since_acq=0.0) -> np.ndarray:
        out = np.zeros(1, SDR_CHAN)
        _check(lib().gnsscorr_sdr_init_chan(_ptr(out), int(sv), int(acq_code_phase),
                                            int(acq_doppler), float(packets_since_acq)),
               "gnsscorr_sdr_init_chan")
        return out[0]

    @staticmethod
    def channel_start(chan, sv, acq_doppler, corr_len=1) -> np.ndarray:
        """Channel::Clear + Channel::Start (objects/channel.cpp:71-170)."""
        out = np.zeros(1, SDR_CHANNEL)
        _check(lib().gnsscorr_sdr_channel_start(_ptr(out), int(chan), int(sv), int(acq_doppler),
                                                int(corr_len)), "gnsscorr_sdr_channel_start")
        return out[0]

    def channel_accum_dev(self, n_ch, n_ms, d_corr, d_chans, d_fb, d_fb_last, d_events,
                          max_events, d_n_events):
        _check(lib().gnsscorr_sdr_channel_accum_dev(self.h, n_ch, n_ms, d_corr, d_chans, d_fb,
                                                    d_fb_last, d_events, max_events, d_n_events),
               "gnsscorr_sdr_channel_accum_dev")

    def channel_accum(self, corr, chans, max_events=4096, all_feedback=True):
        """n_ms Channel::Accum calls per channel: corr (n_ms, n_ch, 6) int32 rows
        (I_E, I_P, I_L, Q_E, Q_P, Q_L); chans SDR_CHANNEL[n_ch] updated in place.
        Returns (feedback SDR_FEEDBACK[n_ms, n_ch] or [n_ch], subframes sorted by (ms, chan))."""
        corr = np.ascontiguousarray(corr, np.int32)
        n_ms, n_ch = corr.shape[0], corr.shape[1]
        assert chans.dtype == SDR_CHANNEL and len(chans) == n_ch
        dev = self.device
        d_c = DevBuf.from_array(corr, dev)
        d_s = DevBuf.from_array(chans, dev)
        d_fb = DevBuf(max(n_ms, 1) * n_ch * SDR_FEEDBACK.itemsize, dev) if all_feedback else None
        d_last = DevBuf(n_ch * SDR_FEEDBACK.itemsize, dev)
        d_ev = DevBuf(max(max_events, 1) * SDR_SUBFRAME.itemsize, dev)
        d_n = DevBuf.from_array(np.zeros(1, np.int32), dev)
        self.channel_accum_dev(n_ch, n_ms, d_c.ptr, d_s.ptr, d_fb.ptr if d_fb else None,
                               d_last.ptr, d_ev.ptr, max_events, d_n.ptr)
        self.sync()
        chans[:] = d_s.download(np.uint8).view(SDR_CHANNEL)
        n = int(d_n.download(np.int32)[0])
        if n > max_events:
            # the kernel keeps whichever max_events subframes won the append race
            raise GnssCorrError(f"channel_accum: {n} subframes exceed max_events={max_events}; "
                                "the kept set would be arbitrary -- raise max_events")
        ev = d_ev.download(np.uint8).view(SDR_SUBFRAME)[:n]
        ev = ev[np.lexsort((ev["chan"], ev["ms"]))]
        if all_feedback:
            fb = d_fb.download(np.uint8).view(SDR_FEEDBACK)[:n_ms * n_ch].reshape(n_ms, n_ch)
        else:
            fb = d_last.download(np.uint8).view(SDR_FEEDBACK)
        return fb, ev, n

    def track_dev(self, d_packets, n_packets, n_rx, n_ch, d_rx, d_states, d_corr, d_chans,
                  d_fb_last, d_log, log_per_ch, d_n_log, d_status, d_events, max_events,
                  d_n_events):
        _check(lib().gnsscorr_sdr_track_dev(self.h, d_packets, n_packets, n_rx, n_ch, d_rx,
                                            d_states, d_corr, d_chans, d_fb_last, d_log,
                                            log_per_ch, d_n_log, d_status, d_events, max_events,
                                            d_n_events), "gnsscorr_sdr_track_dev")

    def track(self, packets, states, corr, chans, rx=None, log_per_ch=0, max_events=4096):
        """The closed loop on the device: packets (n_packets, n_rx, 2048, 2) int16;
        states SDR_CHAN[n_ch], corr SDR_CORR[n_ch], chans SDR_CHANNEL[n_ch] updated in
        place (chans[c] steers states[c]).  Returns dict(fb_last, log SDR_DUMP_REC
        [n_ch, log_per_ch], n_log, status, events sorted by (ms = packet, chan)).
        Raises when a channel's state left the tables (status != 0)."""
        pk = np.ascontiguousarray(packets, np.int16)
        n_packets, n_rx = pk.shape[0], pk.shape[1]
        assert pk.shape[2:] == (2048, 2), pk.shape
        n_ch = len(states)
        assert states.dtype == SDR_CHAN and corr.dtype == SDR_CORR and chans.dtype == SDR_CHANNEL
        assert len(corr) == n_ch and len(chans) == n_ch
        dev = self.device
        d_pk = DevBuf.from_array(pk, dev)
        d_rx = None if rx is None else DevBuf.from_array(np.ascontiguousarray(rx, np.int32), dev)
        d_st, d_c, d_ch = (DevBuf.from_array(a, dev) for a in (states, corr, chans))
        d_last = DevBuf.from_array(np.zeros(n_ch, SDR_FEEDBACK), dev)
        d_log = DevBuf(max(n_ch * log_per_ch, 1) * SDR_DUMP_REC.itemsize, dev)
        d_nlog = DevBuf.from_array(np.zeros(n_ch, np.int32), dev)
        d_stat = DevBuf.from_array(np.zeros(n_ch, np.int32), dev)
        d_ev = DevBuf(max(max_events, 1) * SDR_SUBFRAME.itemsize, dev)
        d_n = DevBuf.from_array(np.zeros(1, np.int32), dev)
        self.track_dev(d_pk.ptr, n_packets, n_rx, n_ch, None if d_rx is None else d_rx.ptr,
                       d_st.ptr, d_c.ptr, d_ch.ptr, d_last.ptr, d_log.ptr, log_per_ch,
                       d_nlog.ptr, d_stat.ptr, d_ev.ptr, max_events, d_n.ptr)
        self.sync()
        status = d_stat.download(np.int32)[:n_ch]
        states[:] = d_st.download(np.uint8).view(SDR_CHAN)
        corr[:] = d_c.download(np.uint8).view(SDR_CORR)
        chans[:] = d_ch.download(np.uint8).view(SDR_CHANNEL)
        if np.any(status != 0):
            c = int(np.flatnonzero(status)[0])
            raise GnssCorrError(f"sdr track: channel {c} stopped (status {int(status[c])}: "
                                "-1 bad receiver index, 1+p state out of the tables at packet p)")
        n = int(d_n.download(np.int32)[0])
        if n > max_events:
            raise GnssCorrError(f"sdr track: {n} subframes exceed max_events={max_events}")
        ev = d_ev.download(np.uint8).view(SDR_SUBFRAME)[:n]
        ev = ev[np.lexsort((ev["chan"], ev["ms"]))]
        log = d_log.download(np.uint8).view(SDR_DUMP_REC)[:n_ch * log_per_ch]
        return dict(fb_last=d_last.download(np.uint8).view(SDR_FEEDBACK),
                    log=log.reshape(n_ch, log_per_ch), n_log=d_nlog.download(np.int32)[:n_ch],
                    status=status, events=ev)

    def accum_dev(self, d_packets, n_jobs, d_jobs, d_out):
        _check(lib().gnsscorr_sdr_accum_dev(self.h, d_packets, n_jobs, d_jobs, d_out),
               "gnsscorr_sdr_accum_dev")

    def correlate(self, packets, states, corr, cb, user=None, rx=None):
        """packets: (n, 2048, 2) int16; states SDR_CHAN[n_ch], corr SDR_CORR[n_ch] in place;
        cb: a C function pointer (int) of gnsscorr_sdr_dump_fn type; user: pointer or None."""
        pk = np.ascontiguousarray(packets, np.int16).reshape(-1, 2048, 2)
        assert states.dtype == SDR_CHAN and corr.dtype == SDR_CORR
        rxa = None if rx is None else np.ascontiguousarray(rx, np.int32)
        _check(lib().gnsscorr_sdr_correlate(self.h, _ptr(pk), pk.shape[0], len(states),
                                            None if rxa is None else _ptr(rxa), _ptr(states),
                                            _ptr(corr), cb, user),
               "gnsscorr_sdr_correlate")

    def sync(self):
        _check(lib().gnsscorr_sdr_corr_sync(self.h), "gnsscorr_sdr_corr_sync")

    @property
    def stream(self) -> int:
        return lib().gnsscorr_sdr_corr_stream(self.h)


# ---------------------------------------------------------------- legacy OSG view
class OSG:
    """The reference's GP2021 register interface, backed by libgnsscorr.

    Accessors mirror osgnss_next_step/src/gp2021/gp2021.c:11-130 (same
    arithmetic, including the NCO word scaling and the `short` truncation of
    from_gps)."""

    MAX_DIGIT = 32

    def __init__(self, samp_rate=16.0e6, gps_if=2.42e6, glonass_if=0.0, sys_clock_mult=5.0,
                 carrier_bits=30, code_bits=29, n_channels=12, use_iq=True,
                 freq_bin_width=1000.0, device=0):
        L = lib()
        _check(L.gnsscorr_osg_configure(samp_rate, gps_if, glonass_if, sys_clock_mult,
                                        carrier_bits, code_bits, n_channels, int(use_iq),
                                        freq_bin_width, device), "gnsscorr_osg_configure")
        self.mult = sys_clock_mult
        self.n_channels = n_channels
        self.carrier_bits = carrier_bits
        self.code_bits = code_bits
        self.REG_read = (C.c_int * 256).in_dll(L, "REG_read")
        self.REG_write = (C.c_int * 256).in_dll(L, "REG_write")

    def get_state(self, n_channels: int = 12) -> np.ndarray:
        st = np.zeros(n_channels, CHAN_STATE)
        _check(lib().gnsscorr_osg_get_state(_ptr(st)), "gnsscorr_osg_get_state")
        return st

    def chan_state(self):
        st = self.get_state(self.n_channels)
        return dict(carrier_phase=st["carrier_phase"].copy(),
                    carrier_cycle=st["carrier_cycle"].copy(),
                    code_phase=st["code_phase"].copy(), half_chip=st["half_chip"].copy(),
                    acc=st["acc"].copy())

    def correlator_init(self, tic_period: float = 0.0):
        lib().correlator_init(tic_period)

    def sim(self, IF: np.ndarray, nsamp: int):
        IF = np.ascontiguousarray(IF, np.int8)
        lib().Sim_GP2021_int(_ptr(IF), nsamp)

    @property
    def gps_carrier_ref(self):
        return C.c_long.in_dll(lib(), "gps_carrier_ref").value

    @property
    def gps_code_ref(self):
        return C.c_long.in_dll(lib(), "gps_code_ref").value

    @property
    def d_freq(self):
        return C.c_long.in_dll(lib(), "d_freq").value

    # --- gp2021.c accessors ---
    def _outpwd(self, add, data):
        self.REG_write[add & 0xFF] = int(data) & 0xFFFF

    def _from_gps(self, add):
        v = self.REG_read[add] & 0xFFFF
        return v - 0x10000 if v >= 0x8000 else v

    def ch_cntl(self, ch, data):
        self._outpwd(ch << 3, data)

    def ch_code_slew(self, ch, data):
        self._outpwd((ch << 3) + 0x84, data)

    def ch_epoch_load(self, ch, data):
        self._outpwd((ch << 3) + 7, data)

    def ch_carrier(self, ch, freq):
        f = int(float(freq << (self.MAX_DIGIT - self.carrier_bits)) * self.mult)
        self._outpwd((ch << 3) + 3, (f >> 16) & 0xFFFF)
        self._outpwd((ch << 3) + 4, f & 0xFFFF)

    def ch_code(self, ch, freq):
        f = int(float(freq << (self.MAX_DIGIT - self.code_bits)) * self.mult)
        self._outpwd((ch << 3) + 5, (f >> 16) & 0xFFFF)
        self._outpwd((ch << 3) + 6, f & 0xFFFF)

    def accum_status(self):
        return self._from_gps(0x82)

    def ch_i_late(self, ch):
        return self._from_gps((ch << 3) + 0x84)

    def ch_q_late(self, ch):
        return self._from_gps((ch << 3) + 0x85)

    def ch_i_prompt(self, ch):
        return self._from_gps((ch << 3) + 0x86)

    def ch_q_prompt(self, ch):
        return self._from_gps((ch << 3) + 0x87)

    def ch_i_early(self, ch):
        return self._from_gps((ch << 3) + 0x88)

    def ch_q_early(self, ch):
        return self._from_gps((ch << 3) + 0x89)
