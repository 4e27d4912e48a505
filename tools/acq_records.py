"""Config-2 throughput with R records per launch (gnsscorr_acq_set_records):
python tools/acq_records.py [steps] [R ...]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import gnsscorr as gc  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 60
Rs = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 1]
for R in Rs:
    ctx, b, meta = bench.acq_setup(0, 0)
    ctx.close()
    IF = np.concatenate([bench.acq_setup(0, r)[2]["IF"] for r in range(R)])
    ctx = gc.AcqCtx(bench.FS, bench.N, device=0, max_freqs=bench.N_BINS,
                    max_blocks=bench.N_BLK * R, max_codes=bench.N_PRN)
    ctx.set_codes(meta["codes"])
    ctx.set_records(R)
    b["d_if"] = gc.DevBuf.from_array(IF, 0)
    b["d_rows"] = gc.DevBuf(R * bench.N_PRN * bench.N_BINS * gc.ACQ_ROW.itemsize, 0)
    b["d_res"] = gc.DevBuf(R * bench.N_PRN * gc.ACQ_RESULT.itemsize, 0)
    for _ in range(3):
        bench.acq_step(ctx, b)
    ctx.sync()
    ev = [gc.Event(0), gc.Event(0)]
    t0 = time.perf_counter()
    for s in range(steps):
        bench.acq_step(ctx, b, ev if s == steps // 2 else None)
    ctx.sync()
    dt = time.perf_counter() - t0
    res = b["d_res"].download(gc.ACQ_RESULT).reshape(R, bench.N_PRN)
    print(f"records {R}: {dt / steps / R * 1e6:.1f} us per search, corr launch "
          f"{ev[0].elapsed_ms(ev[1]) * 1e3:.1f} us, "
          f"{bench.CELLS_PER_SEARCH * steps * R / dt / 1e9:.1f} G cells/s, "
          f"found {sum(int(res[0][p - 1]['metric'] > 2.5) for p in meta['planted'])}/8", flush=True)
    ctx.close()
