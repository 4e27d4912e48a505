"""Per-launch durations of the headline correlation kernel across a timed
region, with and without the host-side found-check between warmup and timing
(events on every step): python tools/acq_step_times.py [steps] [warmup]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import bench  # noqa: E402
from bench import gc  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
warmup = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ctx, b, meta = bench.acq_setup(0, 0, gc.ACQ_F64, bench.ACQ_RECORDS)
for check in (True, False, True, False):
    for _ in range(warmup):
        bench.acq_step(ctx, b)
    ctx.sync()
    if check:   # what run_acq does between warmup and timing
        res = b["d_res"].download(gc.ACQ_RESULT).reshape(bench.ACQ_RECORDS, bench.N_PRN)
        sum(1 for r in range(bench.ACQ_RECORDS) for p in meta["planted"] if res[r][p - 1]["metric"] > 2.5)
    gc.dev_synchronize(0)
    evs = [(gc.Event(0), gc.Event(0)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        bench.acq_step(ctx, b, evs[k])
    ctx.sync()
    dt = time.perf_counter() - t0
    ms = np.array([a.elapsed_ms(z) for a, z in evs])
    print(f"check={check} step_ms={1e3 * dt / steps:.4f} corr_ms first3={np.round(ms[:3], 4).tolist()} "
          f"mean={ms.mean():.4f} median={np.median(ms):.4f} steps0,10={ms[[0, 10]].mean():.4f}", flush=True)
