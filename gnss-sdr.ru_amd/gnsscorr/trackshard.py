"""Tracking channels sharded over ranks (SURVEY 8(e) "Tracking"; BASELINE config 3
scaled out): n_rx receivers x n_ch GP2021 channels, one process per GPU.

Channels are independent (Sim_GP2021_int, osgnss_next_step/src/correlator/
correlator.c:149-316, advances each channel from its own registers and the
shared IF only), so the global channel set is split round-robin: rank r owns
the channels g with g % world == r.  Every rank copies (H2D) the IF streams its
channels read -- with channels spread round-robin that is every stream: the IF
is broadcast by each rank's own host-to-device copy, never over RCCL -- and
runs gnsscorr_track on its GPU with the channels' stream indices remapped to
its local copies.  The only exchange is the gather of the per-channel results
(64 B each) by the caller, over gnsscorr.hostgroup.

`plan()` is pure host logic (tested with the host group on the CPU); `TrackShard` drives
the C-ABI (libgnsscorr.so).
"""
from __future__ import annotations

import numpy as np

from . import NCO_CMD, TRACK_RESULT, DevBuf, TrackCtx


def plan(n_rx: int, n_ch: int, world: int, rank: int):
    """(global channel ids, stream ids this rank must hold, local stream index
    of each of its channels) for round-robin channel sharding."""
    if not (0 <= rank < world) or n_rx < 1 or n_ch < 1:
        raise ValueError("bad shard request")
    mine = [g for g in range(n_rx * n_ch) if g % world == rank]
    streams = sorted({g // n_ch for g in mine})
    local = {s: i for i, s in enumerate(streams)}
    return mine, streams, [local[g // n_ch] for g in mine]


def local_cmds(cmds: np.ndarray, mine, local_stream) -> np.ndarray:
    """This rank's NCO commands: the global rows of its channels, their stream
    field rewritten to the local IF copy they read."""
    out = np.ascontiguousarray(cmds[mine], NCO_CMD).copy()
    out["stream"] = local_stream
    return out


def merge(parts, n_total: int) -> np.ndarray:
    """Per-rank [(global ids, TRACK_RESULT rows)] -> TRACK_RESULT[n_total] in
    global channel order; raises if a channel is missing or duplicated."""
    out = np.zeros(n_total, TRACK_RESULT)
    seen = np.zeros(n_total, np.int32)
    for ids, res in parts:
        ids = np.asarray(ids, np.int64)
        out[ids] = res
        np.add.at(seen, ids, 1)
    if not np.all(seen == 1):
        bad = np.flatnonzero(seen != 1)[:8].tolist()
        raise RuntimeError(f"track merge: channels {bad} missing or duplicated")
    return out


class TrackShard:
    def __init__(self, n_rx: int, n_ch: int, nsamp: int, rank: int = 0, world: int = 1,
                 device: int = 0, samp_rate: float = 16.368e6, iq: bool = True):
        self.n_rx, self.n_ch, self.nsamp, self.iq = n_rx, n_ch, nsamp, iq
        self.mine, self.streams, self.lstream = plan(n_rx, n_ch, world, rank)
        self.bps = 2 if iq else 1                          # bytes per sample
        self.stride = (nsamp + 15) // 16 * 16             # samples per stream (16-B aligned)
        self.device = device
        self.ctx = None
        if not self.mine:       # more ranks than channels: this rank contributes an empty part
            return
        self.ctx = TrackCtx(len(self.mine), iq=iq, device=device, max_nsamp=nsamp,
                            samp_rate=samp_rate)
        self.d_if = DevBuf(max(1, len(self.streams)) * self.stride * self.bps, device)
        self.d_cmds = DevBuf(len(self.mine) * NCO_CMD.itemsize, device)
        self.d_res = DevBuf(len(self.mine) * TRACK_RESULT.itemsize, device)

    def load(self, if_streams: np.ndarray):
        """if_streams: (n_rx, nsamp * bytes-per-sample) int8, one call of every
        receiver's IF; copies (H2D) the streams this rank reads."""
        if self.ctx is None:
            return
        buf = np.zeros((len(self.streams), self.stride * self.bps), np.int8)
        for i, s in enumerate(self.streams):
            row = np.asarray(if_streams[s], np.int8)[:self.nsamp * self.bps]
            buf[i, :len(row)] = row
        self.d_if.upload(buf)

    def step(self, cmds_global: np.ndarray):
        """One Sim_GP2021_int call for this rank's channels (asynchronous)."""
        if self.ctx is None:
            return
        self.d_cmds.upload(local_cmds(cmds_global, self.mine, self.lstream))
        self.ctx.track_dev(self.d_if.ptr, self.stride, self.nsamp, self.d_cmds.ptr,
                           self.d_res.ptr)

    def results(self):
        """(global channel ids, TRACK_RESULT rows) of the last step."""
        if self.ctx is None:
            return [], np.zeros(0, TRACK_RESULT)
        self.ctx.sync()
        return self.mine, self.d_res.download(TRACK_RESULT, len(self.mine))
