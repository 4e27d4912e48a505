"""Debug: look for nonzero fft_buff words in the Channel objects around the
device loop and the replay, repeated in one process."""
import sys
import numpy as np
sys.path[:0] = ["tests", "oracle", "gnss-sdr.ru_amd"]
import gnsscorr as gc
from test_sdr_corr_gpu import _scene
K = 400
pk, chans = _scene(K, n_rx=2)
rx = np.array([c[0] for c in chans], np.int32)
n = len(chans)
for it in range(6):
    ctx = gc.SdrCorrCtx()
    st = np.zeros(n, gc.SDR_CHAN); ch = np.zeros(n, gc.SDR_CHANNEL)
    for c, (r, sv, cp, dop) in enumerate(chans):
        st[c] = ctx.init_chan(sv, cp, dop, 3.0); ch[c] = ctx.channel_start(c, sv, dop, 1)
    ch0 = ch.copy()
    print(it, "ch0 nz", [(c, np.flatnonzero(ch0[c]["fft_buff"])[:4]) for c in range(n) if ch0[c]["fft_buff"].any()])
    out = ctx.track(pk, st, np.zeros(n, gc.SDR_CORR), ch, rx=rx, log_per_ch=2 * K + 2)
    print(it, "track nz", [(c, np.flatnonzero(ch[c]["fft_buff"])[:4]) for c in range(n) if ch[c]["fft_buff"].any()])
    bad = 0
    for c in range(n):
        m = int(out["n_log"][c]); cr = out["log"][c, :m]["corr"]
        rows = np.stack([cr["i"][:, 0], cr["i"][:, 1], cr["i"][:, 2], cr["q"][:, 0], cr["q"][:, 1], cr["q"][:, 2]], 1).astype(np.int32)
        chc = ch0[c:c + 1].copy()
        fb, ev, _ = ctx.channel_accum(rows.reshape(m, 1, 6), chc)
        if chc.tobytes() != ch[c:c + 1].tobytes():
            bad += 1
            print(it, c, "diff", [f for f in gc.SDR_CHANNEL.names if chc[0][f].tobytes() != ch[c][f].tobytes()],
                  np.flatnonzero(chc[0]["fft_buff"])[:4], np.flatnonzero(ch[c]["fft_buff"])[:4])
    print(it, "bad", bad, flush=True)
    del ctx
