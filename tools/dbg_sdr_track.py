"""Debug: which Channel fields differ between the device loop and the replay."""
import sys, os
import numpy as np
sys.path[:0] = ["tests", "oracle", "gnss-sdr.ru_amd"]
import gnsscorr as gc
from test_sdr_corr_gpu import _scene
K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
pk, chans = _scene(K, n_rx=2)
ctx = gc.SdrCorrCtx()
n = len(chans)
st = np.zeros(n, gc.SDR_CHAN); ch = np.zeros(n, gc.SDR_CHANNEL)
for c, (rx, sv, cp, dop) in enumerate(chans):
    st[c] = ctx.init_chan(sv, cp, dop, 3.0); ch[c] = ctx.channel_start(c, sv, dop, 1)
ch0 = ch.copy()
rx = np.array([c[0] for c in chans], np.int32)
out = ctx.track(pk, st, np.zeros(n, gc.SDR_CORR), ch, rx=rx, log_per_ch=2 * K + 2)
for c in range(n):
    m = int(out["n_log"][c]); cr = out["log"][c, :m]["corr"]
    rows = np.stack([cr["i"][:, 0], cr["i"][:, 1], cr["i"][:, 2], cr["q"][:, 0], cr["q"][:, 1], cr["q"][:, 2]], 1).astype(np.int32)
    chc = ch0[c:c + 1].copy()
    fb, ev, _ = ctx.channel_accum(rows.reshape(m, 1, 6), chc)
    diffs = [f for f in gc.SDR_CHANNEL.names if chc[0][f].tobytes() != ch[c][f].tobytes()]
    nz_t = np.flatnonzero(ch[c]["fft_buff"]); nz_r = np.flatnonzero(chc[0]["fft_buff"])
    print(c, m, "count", ch[c]["count"], chc[0]["count"], "diff", diffs, "nz track", nz_t[:8], hex(int(ch[c]["fft_buff"][511])), "nz replay", nz_r[:8], hex(int(chc[0]["fft_buff"][511])))
