"""Full-sky acquisition (BASELINE config 5): 32 GPS PRNs + 14 GLONASS FCHs,
n_bins Doppler bins each, n_ms-ms non-coherent integration, search groups
sharded over ranks (one process per GPU).

Each group (GPS PRN or GLONASS FCH) is searched exactly as
acquisition.sci:95-186 (GPS) / GLONASS acquisition.sci:98-193 does for one
satellite: its own Doppler row set, peak / second peak / metric from its own
winning row.  A group therefore never needs data from another rank: the
shards are disjoint group sets (round-robin, rank r takes groups i with
i % world == r), each rank runs the same HIP kernels on its own GPU, and the
only exchange is the final gather of the per-group results (a few hundred
bytes) -- done by the caller over gnsscorr.hostgroup, not RCCL.

Plumbing over the C-ABI (libgnsscorr.so); the computation is in acq64.hip.
"""
from __future__ import annotations

import numpy as np

from . import (ACQ_NONCOHERENT, ACQ_RESULT, ACQ_ROW, AcqCtx, DevBuf, ca_code, sample_code,
               st_code)

GROUPS = [(0, p) for p in range(1, 33)] + [(1, k) for k in range(-7, 7)]


def shard(n_groups: int, world: int, rank: int) -> list[int]:
    """Round-robin group indices of one rank (balanced to within one group)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return [i for i in range(n_groups) if i % world == rank]


def merge(shards: list[list[tuple]]) -> list[tuple]:
    """Union of per-rank (group_index, system, id, result) lists, in group order;
    raises if a group is missing or duplicated."""
    allr = sorted((r for s in shards for r in s), key=lambda r: r[0])
    idx = [r[0] for r in allr]
    if idx != list(range(len(GROUPS))):
        raise RuntimeError(f"full-sky merge: groups {sorted(set(range(len(GROUPS))) - set(idx))} "
                           f"missing or duplicated")
    return allr


class FullSky:
    """One rank's share of the full-sky search in ONE correlation launch (round 5):
    the GPS and GLONASS IF records sit end to end as two records of one fp64
    context, every group carries its record (gnsscorr_acq_set_group_records), and
    the code table holds the rank's C/A codes plus the ST code.  At world 8 a rank's
    205-246 rows then run as one round of the CUs instead of two launches side by
    side."""

    def __init__(self, fs: float = 16.368e6, n_ms: int = 10, n_bins: int = 41,
                 bin_hz: float = 500.0, if_gps: float = 2.42e6, if_glo: float = 1.0e6,
                 glo_step: float = 0.5625e6, rank: int = 0, world: int = 1, device: int = 0,
                 spc: int = 16):
        self.N = int(round(fs / 1000.0))
        self.fs, self.n_ms, self.n_bins, self.spc, self.device = fs, n_ms, n_bins, spc, device
        self.mine = shard(len(GROUPS), world, rank)
        rel = bin_hz * (np.arange(n_bins) - (n_bins - 1) / 2.0)
        gps = [GROUPS[i][1] for i in self.mine if GROUPS[i][0] == 0]
        glo = [GROUPS[i][1] for i in self.mine if GROUPS[i][0] == 1]
        self.ids = [(0, p) for p in gps] + [(1, k) for k in glo]   # result order
        self.two = bool(gps) and bool(glo)
        codes, freqs, gcode, grec = [], [], [], []
        for p in gps:
            gcode.append(len(codes))
            codes.append(sample_code(ca_code(p), 1.023e6, fs, self.N))
            grec.append(0)
            freqs.append(if_gps + rel)
        if glo:
            st = len(codes)
            codes.append(sample_code(st_code(), 0.511e6, fs, self.N))
            for k in glo:
                gcode.append(st)
                grec.append(1 if self.two else 0)
                freqs.append(if_glo + k * glo_step + rel)
        G = len(self.ids)
        self.freqs = np.concatenate(freqs)
        gf = np.arange(G * n_bins, dtype=np.int32).reshape(G, n_bins)
        dev = device
        self.ctx = AcqCtx(fs, self.N, device=dev, max_freqs=len(self.freqs),
                          max_blocks=n_ms * (2 if self.two else 1), max_codes=len(codes))
        self.ctx.set_codes(np.stack(codes))
        self.d_grec = DevBuf.from_array(np.asarray(grec, np.int32), dev)
        if self.two:
            self.ctx.set_records(2)
            self.ctx.set_group_records(self.d_grec)
        self.G = G
        self.d_if = DevBuf(2 * n_ms * self.N * (2 if self.two else 1), dev)
        self.d_freqs = DevBuf.from_array(self.freqs, dev)
        self.d_gcode = DevBuf.from_array(np.asarray(gcode, np.int32), dev)
        self.d_gfreq = DevBuf.from_array(gf, dev)
        self.d_rows = DevBuf(G * n_bins * ACQ_ROW.itemsize, dev)
        self.d_res = DevBuf(G * ACQ_RESULT.itemsize, dev)

    @property
    def cells(self) -> int:
        """cell-ms this rank searches per run (group x bin x code phase x ms)."""
        return len(self.mine) * self.n_bins * self.N * self.n_ms

    def load(self, if_gps: np.ndarray, if_glo: np.ndarray):
        """Interleaved int8 I,Q records of at least n_ms ms (the GPS and GLONASS front ends)."""
        need = 2 * self.n_ms * self.N
        recs = []
        if any(s_ == 0 for s_, _ in self.ids):
            recs.append(np.ascontiguousarray(if_gps[:need], np.int8))
        if any(s_ == 1 for s_, _ in self.ids):
            recs.append(np.ascontiguousarray(if_glo[:need], np.int8))
        self.d_if.upload(np.concatenate(recs))

    def run(self):
        """Enqueue the search (asynchronous on the context's stream): the forward
        spectra of both records, then one correlation launch for every group."""
        self.ctx.spectra_dev(self.d_if.ptr, self.n_ms, len(self.freqs), self.d_freqs.ptr)
        self.ctx.correlate_dev(self.n_ms, self.d_freqs.ptr, self.G, self.n_bins,
                               self.d_gcode.ptr, self.d_gfreq.ptr, self.d_rows.ptr,
                               self.d_res.ptr, spc=self.spc, mode=ACQ_NONCOHERENT)

    def sync(self):
        self.ctx.sync()

    def results(self) -> list[tuple]:
        """[(group_index, system, prn_or_fch, ACQ_RESULT record)] for this rank's groups."""
        self.sync()
        res = self.d_res.download(ACQ_RESULT, self.G)
        out = [(GROUPS.index(sid), sid[0], sid[1], res[j]) for j, sid in enumerate(self.ids)]
        return sorted(out, key=lambda r: r[0])
