"""Closed-loop OSGPS receiver scenarios at 16.368 Msps (BASELINE configs 1 and 3).

Shared by tests/golden/make_e2e16368_golden.py (which runs the reference
receiver, oracle/_ref/e2e_ref_16368, and stores the trace hash) and
tests/test_e2e_gpu.py (which runs the same receiver on libgnsscorr.so).

The signals are placed in Doppler bins other than the first one searched:
osgpsisr.c:506 starts the FLL/PLL pull-in from chan.carrier_freq, which
ch_acq only sets once the search leaves the 0-Hz bin (:446, :454); a signal
confirmed in that first bin starts pull-in from carrier word 0 and never
locks -- on either correlator (observed with the reference build).
"""
import numpy as np

FS = 16.368e6
NSAMP = 8380                          # SAMP_RATE * interr_int / 1e6 (osgnss_next_step.c:150)
REC = np.dtype([("reg", "<i4", 256), ("state", "<i4", 12), ("carr", "<i8", 12),
                ("code", "<i8", 12), ("nfreq", "<i4", 12), ("codes", "<i4", 12)])
CHANNEL_TRACKING = 4                  # structs.h channel states: 1 acq, 2 confirm, 3 pull-in

SCENARIOS = {
    # BASELINE config 1: PRN 1, one channel, acquire + track
    "config1": dict(calls=32000, prns=[1], seed=0x5EED0001,
                    sigs=[dict(system=0, prn=1, code_phase=412.0, doppler=1000.0, cn0=50.0,
                               data_bits=1)]),
    # BASELINE config 3: 12 channels, 8 of them with a signal
    "config3": dict(calls=50000, prns=[1, 3, 7, 11, 14, 17, 19, 21, 24, 27, 28, 31],
                    seed=0x5EED0003,
                    sigs=[dict(system=0, prn=p, code_phase=cp, doppler=d, cn0=50.0, data_bits=1)
                          for p, cp, d in [(1, 412.0, 1000.0), (3, 35.5, 1150.0),
                                           (7, 220.0, 850.0), (11, 90.25, 1250.0),
                                           (14, 600.0, 920.0), (17, 18.0, 1080.0),
                                           (19, 333.0, 780.0), (21, 150.0, 1200.0)]]),
}


def make_if(gc, name):
    s = SCENARIOS[name]
    return gc.ifgen(NSAMP * s["calls"], s["sigs"], fs=FS, if_gps=2.42e6, seed=s["seed"])


def summary(trace: bytes, n_ch: int):
    """Per channel: first call in CHANNEL_TRACKING (-1 if never), seconds held to the end."""
    tr = np.frombuffer(trace, REC)
    out = []
    for ch in range(n_ch):
        st = tr["state"][:, ch]
        i4 = np.flatnonzero(st == CHANNEL_TRACKING)
        if len(i4) and np.all(st[i4[0]:] == CHANNEL_TRACKING):
            out.append((int(i4[0]), (len(tr) - int(i4[0])) * NSAMP / FS))
        else:
            out.append((-1, 0.0))
    return out
