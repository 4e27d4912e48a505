"""C_s = 1 int8 tracking, single-call launches, two IF layouts of the same bytes:
python tools/trk_callmajor.py [calls]
* stream-major: stream s holds all calls (call k at s*K*nsamp + k*nsamp samples), the
  layout bench.py's cs1 lines replay;
* call-major: call k holds all streams (stream s at k*C*nsamp + s*nsamp), the layout of a
  front end that lands one millisecond of every channel as one block.
Prints kernel us per 3072 channel-ms for each (HIP events around the timed calls)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bench import gc  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
warmup = 5
K = steps + warmup
NS = bench.TRACK_NS
C = int(os.environ.get("TRK_C", str(bench.TRACK_C1)))
rng = np.random.default_rng(17)
d_if = gc.DevBuf(C * K * NS * 2, 0)
d_if.fill_if2(0x5EED000B)
cmd1 = bench._track_cmds(rng, C, np.arange(C))
d_cmds = gc.DevBuf.from_array(cmd1, 0)
d_res = gc.DevBuf(C * gc.TRACK_RESULT.itemsize, 0)
for name, stride, step_b in (("stream_major", K * NS, NS * 2), ("call_major", NS, C * NS * 2),
                             ("stream_major", K * NS, NS * 2), ("call_major", NS, C * NS * 2)):
    ctx = gc.TrackCtx(C, iq=True, device=0, max_nsamp=NS, samp_rate=bench.FS)
    ctx.set_layout(True)
    for k in range(warmup):
        ctx.track_dev(d_if.ptr + k * step_b, stride, NS, d_cmds.ptr, d_res.ptr, 0, ctx.next_tic(NS))
    e0, e1 = gc.Event(0), gc.Event(0)
    e0.record(ctx.stream)
    for k in range(warmup, K):
        ctx.track_dev(d_if.ptr + k * step_b, stride, NS, d_cmds.ptr, d_res.ptr, 0, ctx.next_tic(NS))
    e1.record(ctx.stream)
    ctx.sync()
    ms = e0.elapsed_ms(e1) / steps
    print(name, "ms per call %.4f" % ms, "us per 3072 channel-ms %.2f" % (ms * 1e3 * 3072 / C),
          flush=True)
    ctx.close()
