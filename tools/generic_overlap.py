"""Does the generic engine's search leave the GPU idle enough for a second one to
overlap?  Times K config-2 searches at 38.192 Msps on one context, then K searches
on each of two contexts (two HIP streams) issued alternately: prints ms per search."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnss-sdr.ru_amd"))
import numpy as np  # noqa: E402
import gnsscorr as gc  # noqa: E402

FS, NB, NPRN, NBIN, K = 38.192e6, 2, 32, 41, 20
N = int(round(FS / 1000.0))
SPC = int(round(FS / 1.023e6))


def make(dev=0):
    ctx = gc.AcqCtx(FS, N, device=dev, max_freqs=NBIN, max_blocks=NB, max_codes=NPRN)
    ctx.set_prn_codes(np.arange(1, NPRN + 1, dtype=np.int32))
    IF = gc.ifgen(NB * N, [dict(system=0, prn=5, code_phase=300.0, doppler=-1500.0, cn0=49.0,
                                data_bits=1)], fs=FS, seed=11)
    freqs = 2.42e6 - 10000.0 + 500.0 * np.arange(NBIN)
    b = dict(d_if=gc.DevBuf.from_array(IF, dev), d_f=gc.DevBuf.from_array(freqs, dev),
             d_gc=gc.DevBuf.from_array(np.arange(NPRN, dtype=np.int32), dev),
             d_gf=gc.DevBuf.from_array(np.tile(np.arange(NBIN, dtype=np.int32), NPRN), dev),
             d_rows=gc.DevBuf(NPRN * NBIN * gc.ACQ_ROW.itemsize, dev),
             d_res=gc.DevBuf(NPRN * gc.ACQ_RESULT.itemsize, dev))
    return ctx, b


def search(ctx, b):
    ctx.spectra_dev(b["d_if"].ptr, NB, NBIN, b["d_f"].ptr)
    ctx.correlate_dev(NB, b["d_f"].ptr, NPRN, NBIN, b["d_gc"].ptr, b["d_gf"].ptr, spc=SPC)
    ctx.select_dev(NPRN, NBIN, b["d_f"].ptr, b["d_gf"].ptr, b["d_rows"].ptr, b["d_res"].ptr)


A, B = make(), make()
for _ in range(3):
    search(*A)
    search(*B)
A[0].sync()
B[0].sync()
t0 = time.perf_counter()
for _ in range(K):
    search(*A)
A[0].sync()
one = (time.perf_counter() - t0) * 1e3 / K
t0 = time.perf_counter()
for _ in range(K):
    search(*A)
    search(*B)
A[0].sync()
B[0].sync()
two = (time.perf_counter() - t0) * 1e3 / (2 * K)
print(json.dumps({"ms_per_search_one_stream": round(one, 4), "ms_per_search_two_streams": round(two, 4)}))
