"""Tracking kernel scaling probe: kernel time vs channel count and call length."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnss-sdr.ru_amd"))
import gnsscorr as gc  # noqa: E402


def run(C, ns, steps=20, warm=3, ch_per_rx=12):
    rx = (C + ch_per_rx - 1) // ch_per_rx
    K = steps + warm
    stride = K * ns
    d_if = gc.DevBuf(rx * stride * 2)
    d_if.fill_if2(5)
    rng = np.random.default_rng(1)
    cmd = np.zeros(C, gc.NCO_CMD)
    cmd["prn"] = rng.integers(1, 33, C)
    cmd["stream"] = np.arange(C) // ch_per_rx
    cmd["carrier_incr"] = 635008600 + rng.integers(-262000, 262000, C) * 20
    cmd["code_incr"] = 6710886 * 40 + rng.integers(-10, 10, C)
    cmd["epoch_load"] = -1
    d_c = gc.DevBuf.from_array(np.tile(cmd, K))
    d_r = gc.DevBuf(K * C * gc.TRACK_RESULT.itemsize)
    ctx = gc.TrackCtx(C, iq=True, max_nsamp=ns, samp_rate=16.368e6)
    ctx.replay_dev(d_if.ptr, stride, ns, warm, d_c.ptr, d_r.ptr)
    e0, e1 = gc.Event(), gc.Event()
    e0.record(ctx.stream)
    ctx.replay_dev(d_if.ptr + warm * ns * 2, stride, ns, steps,
                   d_c.ptr + warm * C * gc.NCO_CMD.itemsize,
                   d_r.ptr + warm * C * gc.TRACK_RESULT.itemsize)
    e1.record(ctx.stream)
    ctx.sync()
    ms = e0.elapsed_ms(e1) / steps
    print(f"C={C:6d} ns={ns:6d} kernel {ms * 1e3:8.1f} us  {C * ns / ms / 1e6:8.1f} Msamp/ms",
          flush=True)


for C in (1024, 3072, 12288):
    run(C, 16368)
for ns in (8384,):
    run(3072, ns)
