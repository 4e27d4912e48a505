"""Config-2 searches with 1, 2 or 3 contexts in flight (one HIP stream each):
python tools/acq_inflight.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gnsscorr as gc  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
for k in (1, 2, 3, 1):
    ctxs = [bench.acq_setup(0, 0) for _ in range(k)]
    for _ in range(3):
        for c, b, _m in ctxs:
            bench.acq_step(c, b)
    for c, _b, _m in ctxs:
        c.sync()
    gc.dev_synchronize(0)
    t0 = time.perf_counter()
    for s in range(steps):
        c, b, _m = ctxs[s % k]
        bench.acq_step(c, b)
    for c, _b, _m in ctxs:
        c.sync()
    gc.dev_synchronize(0)
    dt = time.perf_counter() - t0
    ok = all(sum(1 for p in m["planted"] if b["d_res"].download(gc.ACQ_RESULT)[p - 1]["metric"] > 2.5)
             == len(m["planted"]) for _c, b, m in ctxs)
    print(f"in flight {k}: {dt / steps * 1e6:.1f} us per search, "
          f"{bench.CELLS_PER_SEARCH * steps / dt / 1e9:.1f} G cells/s, planted found: {ok}", flush=True)
    del ctxs
