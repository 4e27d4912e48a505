"""Debug: multi-call replay vs sequential single calls, per call index."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gnss-sdr.ru_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import gnsscorr as gpu
import osg_scenarios as S
from test_track_gpu import _random_cmds
rng = np.random.default_rng(9)
C, K, nsamp = 256, 4, 16368
IF = S.synth_if(nsamp * K, 77, [(5, 10, 0, 3)])
cmds = _random_cmds(rng, K, C, 1)
seq = gpu.TrackCtx(C, max_nsamp=nsamp)
seq_res, seq_st = [], []
for k in range(K):
    r, _ = seq.track(IF[k * nsamp * 2:(k + 1) * nsamp * 2], nsamp, cmds[k])
    seq_res.append(r)
    seq_st.append(seq.get_state())
for KK in (1, 2, K):
    rep = gpu.TrackCtx(C, max_nsamp=nsamp)
    d_if = gpu.DevBuf.from_array(IF)
    d_cmds = gpu.DevBuf.from_array(cmds)
    d_res = gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize)
    rep.replay_dev(d_if.ptr, 0, nsamp, KK, d_cmds.ptr, d_res.ptr)
    rep.sync()
    got = d_res.download(gpu.TRACK_RESULT).reshape(K, C)
    st = rep.get_state()
    for k in range(KK):
        bad = np.flatnonzero((got[k]["dump"] != seq_res[k]["dump"]).any(1) |
                             (got[k]["n_dumps"] != seq_res[k]["n_dumps"]))
        print(f"K={KK} call {k}: {len(bad)} channels differ", bad[:8])
    for f in ("carrier_phase", "code_phase", "half_chip", "acc", "ms_counter"):
        print("  state", f, "equal" if np.array_equal(st[f], seq_st[KK - 1][f]) else "DIFFERS")
# detail: one differing channel of call 1 (K=2)
rep = gpu.TrackCtx(C, max_nsamp=nsamp)
d_if = gpu.DevBuf.from_array(IF)
d_cmds = gpu.DevBuf.from_array(cmds)
d_res = gpu.DevBuf(K * C * gpu.TRACK_RESULT.itemsize)
rep.replay_dev(d_if.ptr, 0, nsamp, 2, d_cmds.ptr, d_res.ptr)
rep.sync()
got = d_res.download(gpu.TRACK_RESULT).reshape(K, C)
bad = np.flatnonzero((got[1]["dump"] != seq_res[1]["dump"]).any(1))
for b in bad[:6]:
    print("ch", b, "got", got[1]["dump"][b], "want", seq_res[1]["dump"][b], "diff", got[1]["dump"][b] - seq_res[1]["dump"][b],
          "nd", got[1]["n_dumps"][b], seq_res[1]["n_dumps"][b])
# tiny launch: 4 channels
C2 = 4
seq2 = gpu.TrackCtx(C2, max_nsamp=nsamp)
rs = []
for k in range(2):
    r, _ = seq2.track(IF[k * nsamp * 2:(k + 1) * nsamp * 2], nsamp, cmds[k][:C2])
    rs.append(r)
rep2 = gpu.TrackCtx(C2, max_nsamp=nsamp)
c2 = np.ascontiguousarray(cmds[:2, :C2])
d_c2 = gpu.DevBuf.from_array(c2)
d_r2 = gpu.DevBuf(2 * C2 * gpu.TRACK_RESULT.itemsize)
rep2.replay_dev(d_if.ptr, 0, nsamp, 2, d_c2.ptr, d_r2.ptr)
rep2.sync()
g2 = d_r2.download(gpu.TRACK_RESULT).reshape(2, C2)
print("C=4 call1 equal:", np.array_equal(g2[1]["dump"], rs[1]["dump"]), g2[1]["dump"][:2], rs[1]["dump"][:2])
