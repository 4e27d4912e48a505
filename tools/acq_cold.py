"""Where a context's first code spectra and first search spend their time.

python tools/acq_cold.py  -> one JSON line: milliseconds for gnsscorr_acq_create,
the first and a later set_prn_codes (+ sync), the first and a later config-2
search (spectra + correlate + select + sync), for the process's first context
and for a second one created after it (code objects already loaded).
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnss-sdr.ru_amd"))
import gnsscorr as gc  # noqa: E402

FS, N, NB, NPRN, NBIN = 16.368e6, 16368, 2, 32, 41


def one_context(dev=0):
    ms = lambda t0: round((time.perf_counter() - t0) * 1e3, 4)  # noqa: E731
    out = {}
    t0 = time.perf_counter()
    ctx = gc.AcqCtx(FS, N, device=dev, max_freqs=NBIN, max_blocks=NB, max_codes=NPRN)
    out["create_ms"] = ms(t0)
    ids = np.arange(1, NPRN + 1, dtype=np.int32)
    for k in ("codes_first_ms", "codes_second_ms"):
        t0 = time.perf_counter()
        ctx.set_prn_codes(ids)
        ctx.sync()
        out[k] = ms(t0)
    IF = gc.ifgen(NB * N, [dict(system=0, prn=3, code_phase=100.0, doppler=1000.0, cn0=49.0,
                                data_bits=1)], fs=FS, seed=7)
    freqs = 2.42e6 - 10000.0 + 500.0 * np.arange(NBIN)
    d_if = gc.DevBuf.from_array(IF, dev)
    d_f = gc.DevBuf.from_array(freqs, dev)
    d_gc = gc.DevBuf.from_array(np.arange(NPRN, dtype=np.int32), dev)
    d_gf = gc.DevBuf.from_array(np.tile(np.arange(NBIN, dtype=np.int32), NPRN), dev)
    d_rows = gc.DevBuf(NPRN * NBIN * gc.ACQ_ROW.itemsize, dev)
    d_res = gc.DevBuf(NPRN * gc.ACQ_RESULT.itemsize, dev)
    for k in ("search_first_ms", "search_second_ms"):
        t0 = time.perf_counter()
        ctx.spectra_dev(d_if.ptr, NB, NBIN, d_f.ptr)
        ctx.correlate_dev(NB, d_f.ptr, NPRN, NBIN, d_gc.ptr, d_gf.ptr)
        ctx.select_dev(NPRN, NBIN, d_f.ptr, d_gf.ptr, d_rows.ptr, d_res.ptr)
        ctx.sync()
        out[k] = ms(t0)
    res = d_res.download(gc.ACQ_RESULT)
    out["prn3_found"] = bool(res[2]["metric"] > 2.5)
    return out


if __name__ == "__main__":
    print(json.dumps({"first_context": one_context(), "second_context": one_context(),
                      "lib": os.environ.get("GNSSCORR_LIB", "in-tree")}))
