"""Debug helper: osg_track2_kernel vs osg_track_kernel (GNSSCORR_TRACK_V1=1) on the same
random channel states and commands; prints the channels that differ."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "gnss-sdr.ru_amd"))
import gnsscorr as gc  # noqa: E402

nsamp = int(sys.argv[1]) if len(sys.argv) > 1 else 8380
packed = len(sys.argv) > 2 and sys.argv[2] == "packed"
mode = sys.argv[3] if len(sys.argv) > 3 else "code"
C = 64
rng = np.random.default_rng(5)
IF = rng.choice(np.array([-3, -1, 1, 3], np.int8), 2 * nsamp * C)
if mode == "zeroIQ":
    IF[1::2] = 0
st0 = np.zeros(C, gc.CHAN_STATE)
st0["carrier_phase"] = rng.integers(0, 2**32, C, dtype=np.uint64).astype(np.uint32)
st0["code_phase"] = rng.integers(0, 2**32, C, dtype=np.uint64).astype(np.uint32)
st0["half_chip"] = rng.integers(0, 2046, C)
st0["half_chip"][:16] = rng.integers(1500, 2046, 16)
cmd = np.zeros(C, gc.NCO_CMD)
cmd["prn"] = rng.integers(1, 33, C)
cmd["stream"] = np.arange(C)
cmd["carrier_incr"] = rng.integers(0, 2**32, C, dtype=np.uint64).astype(np.uint32)
cmd["code_incr"] = (2**31 / 8.0 * (1 + rng.uniform(-1e-3, 1e-3, C))).astype(np.uint32)
if mode == "nocode":
    cmd["code_incr"] = 0
if mode == "nocarrier":
    cmd["carrier_incr"] = 0
    st0["carrier_phase"] = 0
cmd["epoch_load"] = -1
out = {}
for v in ("1", "0"):
    os.environ["GNSSCORR_TRACK_V1"] = v
    ctx = gc.TrackCtx(C, iq=True, max_nsamp=nsamp, samp_rate=16.0e6, packed=packed)
    ctx.set_state(st0)
    src = gc.pack2(IF) if packed else IF
    res, _ = ctx.track(src, nsamp, cmd, n_streams=C, stream_stride=nsamp)
    out[v] = (res.copy(), ctx.get_state().copy())
    ctx.close()
r1, s1 = out["1"]
r0, s0 = out["0"]
bad = 0
for c in range(C):
    d = (r1["n_dumps"][c] != r0["n_dumps"][c] or (r1["dump"][c] != r0["dump"][c]).any()
         or (s1["acc"][c] != s0["acc"][c]).any())
    if d:
        bad += 1
        if bad <= 12:
            print(c, "hc0", st0["half_chip"][c], "nd", r1["n_dumps"][c], r0["n_dumps"][c],
                  "dump v1", r1["dump"][c].tolist(), "v2", r0["dump"][c].tolist(),
                  "acc v1", s1["acc"][c].tolist(), "v2", s0["acc"][c].tolist(),
                  "sum v1", (r1["dump"][c].astype(np.int64) + s1["acc"][c]).tolist(),
                  "v2", (r0["dump"][c].astype(np.int64) + s0["acc"][c]).tolist())
print(sys.argv[1:], "channels differing:", bad, "of", C)
