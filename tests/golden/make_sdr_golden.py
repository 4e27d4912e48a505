"""Generate tests/golden/sdr_*.npz from the REFERENCE GPS-SDR primitives.

oracle/_ref/libsdr_ref.so is the reference's simd/x86.cpp, objects/fft.cpp and
accessories/misc.cpp compiled with -DNO_SIMD from /root/reference (make -C
oracle ref), plus PRN_Codes from accessories/prn_codes.h.  Stored:
  sdr_prn_codes.npz   the PRN_Codes table (51 x 2048 x (re, im) int16)
  sdr_acq.npz         input buffers (2048 CPX each, deterministic) and the
                      reference doPrepIF + doAcqStrong results for sv 0..31
  sdr_fft.npz         int16 FFT known answers (forward / inverse, rank masks,
                      incl. inputs large enough to exercise the int16 wrap)
  sdr_corr.npz        tracking correlator: SHA-256 of the 3001 x 4096 carrier
                      wipe-off table built with the reference sine_gen, the
                      code_gen chips of sv 0..31, and Correlator::Accum known
                      answers (x86_cmulsc + x86_prn_accum_new) on random jobs
  sdr_frontend.npz    downsample() (accessories/misc.cpp:174-197) known answers
                      from the reference build at the receiver's source rates
  sdr_acq_mw.npz      medium / weak acquisition (doPrepIF at 10 / 310 ms,
                      doAcqMedium, doAcqWeak, acquisition.cpp:191-236,309-570)
                      over the reference primitives, one session: medium on a
                      fresh object, weak, then medium again (it reads rows the
                      weak prep left, the reference's 20-row stride)
Usage:  python tests/golden/make_sdr_golden.py [mw]   (mw: only sdr_acq_mw.npz)
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import sdr_oracle as S  # noqa: E402

SCENES = [  # (seed, amp_noise, signals)
    (1, 2.0, [dict(prn=5, code_phase=300.0, doppler=2250.0, amp=1.0),
              dict(prn=17, code_phase=800.3, doppler=-4100.0, amp=0.8)]),
    (2, 4.0, [dict(prn=1, code_phase=10.5, doppler=-12300.0, amp=1.5),
              dict(prn=32, code_phase=1000.0, doppler=7777.0, amp=1.2),
              dict(prn=12, code_phase=511.0, doppler=0.0, amp=1.0)]),
    (3, 40.0, [dict(prn=24, code_phase=77.0, doppler=14000.0, amp=30.0)]),   # large levels
]


MW_SIGS = [dict(prn=5, code_phase=300.0, doppler=2250.0, amp=0.45),
           dict(prn=17, code_phase=800.3, doppler=-4100.0, amp=0.15),
           dict(prn=26, code_phase=10.0, doppler=1000.0, amp=0.09)]
MW_WEAK_SVS = [4, 16, 25, 9]


def make_mw(ref, out):
    """Medium / weak session fixture (see module docstring)."""
    buf = S.make_long_buffer(MW_SIGS, 310, seed=21, amp_noise=1.5)
    sess = S.RefAcqSession(ref)
    svs = np.arange(32)
    sess.prep(buf, 10)
    med0 = sess.search("medium", svs)
    sess.prep(buf, 310)
    weak = sess.search("weak", MW_WEAK_SVS, -5000, 5000)
    sess.prep(buf, 10)
    med1 = sess.search("medium", svs, -7000, 3000)
    np.savez_compressed(os.path.join(out, "sdr_acq_mw.npz"), buffer=buf.astype(np.int8),
                        medium_fresh=med0, weak_svs=np.array(MW_WEAK_SVS, np.int32), weak=weak,
                        medium_after_weak=med1, fif=np.array(S.IF_SDR))
    for name, r in (("medium", med0), ("weak", weak), ("medium2", med1)):
        top = sorted(r, key=lambda v: -int(v["magnitude"]))[:3]
        print(name, [(int(v["sv"]) + 1, int(v["code_phase"]), int(v["doppler"]),
                      int(v["magnitude"])) for v in top])


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    if sys.argv[1:] == ["mw"]:
        make_mw(S.RefSDR(), os.path.dirname(os.path.abspath(__file__)))
        return
    ref = S.RefSDR()
    out = os.path.dirname(os.path.abspath(__file__))
    np.savez_compressed(os.path.join(out, "sdr_prn_codes.npz"), prn_codes=ref.prn_codes())
    bufs = np.stack([S.make_buffer(sig, seed=seed, amp_noise=a) for seed, a, sig in SCENES])
    svs = np.arange(32)
    res = np.stack([ref.acq_strong(b, svs) for b in bufs])
    res_narrow = np.stack([ref.acq_strong(b, svs, -3000, 5000) for b in bufs])
    np.savez_compressed(os.path.join(out, "sdr_acq.npz"), buffers=bufs, svs=svs, res=res,
                        res_narrow=res_narrow, fif=np.array(S.IF_SDR))
    rng = np.random.default_rng(11)
    xs = np.stack([rng.integers(-a, a + 1, (2048, 2)) for a in (3, 300, 20000)]).astype(np.int16)
    fwd = np.stack([ref.fft(x, False, S.R1) for x in xs])
    inv = np.stack([ref.fft(x, True, S.R2) for x in xs])
    np.savez_compressed(os.path.join(out, "sdr_fft.npz"), x=xs, fwd_r1=fwd, inv_r2=inv)
    # tracking correlator
    import hashlib
    car = np.stack([ref.sine_gen(np.float32(-38400.0) - np.float32(k) * np.float32(10.0), n=4096)
                    for k in range(-1500, 1501)])
    chips = np.stack([ref.code_gen(sv) for sv in range(32)]).astype(np.uint8)
    o = S.OracleSdrCorr()
    jobs, data, exp = [], [], []
    for it in range(48):
        amp = (3, 300, 32767)[it % 3]
        d = rng.integers(-amp, amp + 1, (2048, 2)).astype(np.int16)
        sb, so, n = int(rng.integers(0, 3001)), int(rng.integers(0, 2048)), int(rng.integers(0, 2049))
        sv, cb, co = int(rng.integers(0, 32)), rng.integers(0, 101, 3), rng.integers(0, 2048, 3)
        codes = [o.code[sv, cb[k], co[k]:co[k] + n] for k in range(3)]
        exp.append(ref.accum(d, car[sb, so:so + n], codes[0], codes[1], codes[2], n))
        jobs.append([0, 0, n, sv, sb, so, *cb, *co])
        data.append(d)
    np.savez_compressed(os.path.join(out, "sdr_corr.npz"),
                        carrier_sha256=np.array(hashlib.sha256(car.tobytes()).hexdigest()),
                        chips=chips, jobs=np.array(jobs, np.int32), data=np.stack(data),
                        expected=np.stack(exp))
    # sample front end: downsample() at the USRP rates of Resample_USRP_V1
    # (gps_source.cpp:823-856: f_sample / decimate = 4.0, 4.096 and 8.0 Msps)
    fe_src, fe_out, fe_rates = [], [], []
    for k, fs in enumerate((4.0e6, 4.096e6, 8.0e6, 2.5e6)):
        n = int(fs / 1000) + 7 * k
        src = rng.integers(-2000, 2001, (n, 2)).astype(np.int16)
        fe_src.append(np.pad(src, ((0, 8200 - n), (0, 0))))
        o = ref.downsample(src, 2.048e6, fs)
        fe_out.append(np.pad(o, ((0, 4200 - len(o)), (0, 0))))
        fe_rates.append((fs, n, len(o)))
    np.savez_compressed(os.path.join(out, "sdr_frontend.npz"), src=np.stack(fe_src),
                        out=np.stack(fe_out), rates=np.array(fe_rates))
    make_mw(ref, out)
    for k, r in enumerate(res):
        print("scene", k, [(int(v["sv"]) + 1, int(v["code_phase"]), int(v["doppler"]),
                            int(v["magnitude"])) for v in r if v["magnitude"] > 0][:3])


if __name__ == "__main__":
    main()
