"""One tracking layout alone, for PMC passes: python tools/trk_layout.py <layout> [calls]
layout: cs1_int8 | cs1_packed2 | rx12_int8 | rx12_packed2 (3072 channels, 1-ms calls at
16.368 Msps, distinct IF every call, the NCO schedule of bench.py's tracking lines)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bench import gc  # noqa: E402

layout = sys.argv[1]
steps = bench._track_steps(int(sys.argv[2]) if len(sys.argv) > 2 else 20)
warmup = bench.TRACK_CPL   # one launch (bench.py's tracking lines: TRACK_CPL calls per launch)
K = steps + warmup
packed = layout.endswith("packed2")
cs1 = layout.startswith("cs1")
C = int(os.environ.get("TRK_C", str(bench.TRACK_C1)))   # channels (TRK_C: other launch sizes)
n_streams = C if cs1 else C // 12
stride = K * bench.TRACK_NS
rng = np.random.default_rng(17)
d_if = gc.DevBuf(n_streams * stride * 2 // (4 if packed else 1), 0)
d_if.fill_if2(0x5EED000B)
cmd1 = bench._track_cmds(rng, C, np.arange(C) if cs1 else np.repeat(np.arange(n_streams), 12))
d_cmds = gc.DevBuf.from_array(np.tile(cmd1, K), 0)
d_res = gc.DevBuf(K * C * gc.TRACK_RESULT.itemsize, 0)
ctx = gc.TrackCtx(C, iq=True, device=0, max_nsamp=bench.TRACK_NS, samp_rate=bench.FS,
                  packed=packed)
dt, kms, res = bench._replay_timed(bench.Dist(), 0, ctx, d_if, stride, ctx.if_bytes(bench.TRACK_NS),
                                   d_cmds, d_res, C, steps, warmup)
print(layout, "kernel ms per call %.4f" % kms, "channels", C,
      "us per 3072 channel-ms %.2f" % (kms * 1e3 * 3072 / C))
