"""CPU: cross-pin of the Scilab-path oracle on shared planted scenes.

acquisition.sci cannot be executed here (no Scilab), so oracle/acq_oracle.py is
"parity unpinned" against a Scilab run.  SURVEY 8(c)
names the only available pin: cross-agreement with the reference's own integer
GPS-SDR acquisition on the same physical signal.  Each scene plants one C/A
signal (PRN, code phase tau at t = 0, Doppler) and is searched twice:

  * acquisition.sci semantics (fp64 restatement, the oracle of the headline
    GPU path) on a 16.368 Msps, 2.42 MHz IF record from gnsscorr_ifgen:
    code start = codePhase - 1 samples (SCI/GPS/L1/acquisition.sci:141-169),
    Doppler = frequencyBin - IF;
  * Acquisition::doAcqStrong of the GPS-SDR receiver COMPILED FROM THE
    REFERENCE SOURCES (oracle/_ref/libsdr_ref.so: x86.cpp, fft.cpp, misc.cpp
    -DNO_SIMD, prn_codes.h) on the same signal generated at 2.048 Msps and
    38.4 kHz IF: code start = 2048 - code_phase samples (code_phase = 2048 - argmax),
    Doppler = lcv*1000 + lcv2*250
    (SDR/objects/acquisition.cpp:244-301).

The two must agree on the code start to within one 2.048 Msps sample (the
integer path's resolution) and on the Doppler to within one 500-Hz bin, and both
must sit at the planted truth.  A wrong sign convention, bin map, 1-based index
or circular-shift direction in the restatement fails this.
"""
import numpy as np
import pytest

import acq_oracle as A
import sdr_oracle as S

FS1, N1, IF1 = 16.368e6, 16368, 2.42e6
SCENES = [(3, 100.0, 1750.0), (11, 512.25, -3250.0), (22, 900.6, 4250.0), (31, 7.3, -500.0)]


@pytest.fixture(scope="module")
def ref():
    if not S.have_ref():
        pytest.skip("reference GPS-SDR build absent (oracle/_ref/libsdr_ref.so)")
    return S.RefSDR()


@pytest.mark.parametrize("prn,tau,dop", SCENES)
def test_scilab_path_agrees_with_reference_gps_sdr(gc, ref, prn, tau, dop):
    # acquisition.sci path (config-2 grid: 41 bins at 500 Hz around the IF)
    IF = gc.ifgen(2 * N1, [dict(system=0, prn=prn, code_phase=tau, doppler=dop, cn0=48.0)],
                  fs=FS1, seed=0x5EED0030 + prn)
    freqs = IF1 - 10000.0 + 500.0 * np.arange(41)
    code = A.make_ca_table_row(prn, FS1)[None]
    res = A.acquire(IF, FS1, code, freqs, np.arange(41)[None])[0]
    start1 = (res["code_phase"] - 1) / FS1                      # seconds into the 1-ms period
    dop1 = freqs[res["bin"]] - IF1
    # the reference's integer path on the same signal at 2.048 Msps
    buf = S.make_buffer([dict(prn=prn, code_phase=tau, doppler=dop, amp=1.5)], n=S.N,
                        seed=0x5EED0040 + prn, amp_noise=2.0)
    r = ref.acq_strong(buf, [prn - 1])[0]
    start2 = ((S.N - r["code_phase"]) % S.N) / S.FS           # code_phase = 2048 - argmax
    dop2 = float(r["doppler"])
    # both at the truth, and with each other
    truth = ((1023.0 - tau) % 1023.0) / 1.023e6
    period = 1e-3

    def circ(a, b):
        d = abs(a - b) % period
        return min(d, period - d)

    ts2 = 1.0 / S.FS
    assert circ(start1, truth) <= 1.0 / FS1 + 1e-9, (start1, truth)
    assert circ(start2, truth) <= ts2 + 1e-9, (start2, truth)
    assert circ(start1, start2) <= ts2 + 1.0 / FS1 + 1e-9, (start1, start2)
    assert abs(dop1 - dop) <= 250.0 and abs(dop2 - dop) <= 250.0, (dop1, dop2, dop)
    assert abs(dop1 - dop2) <= 500.0
