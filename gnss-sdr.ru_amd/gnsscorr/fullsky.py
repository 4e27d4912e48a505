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
bytes) -- done by the caller over gloo, not RCCL.

Plumbing over the C-ABI (libgnsscorr.so); the computation is in acq.hip.
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
    def __init__(self, fs: float = 16.368e6, n_ms: int = 10, n_bins: int = 41,
                 bin_hz: float = 500.0, if_gps: float = 2.42e6, if_glo: float = 1.0e6,
                 glo_step: float = 0.5625e6, rank: int = 0, world: int = 1, device: int = 0,
                 spc: int = 16):
        self.N = int(round(fs / 1000.0))
        self.fs, self.n_ms, self.n_bins, self.spc, self.device = fs, n_ms, n_bins, spc, device
        self.mine = shard(len(GROUPS), world, rank)
        rel = bin_hz * (np.arange(n_bins) - (n_bins - 1) / 2.0)
        self.parts = []
        gps = [GROUPS[i][1] for i in self.mine if GROUPS[i][0] == 0]
        glo = [GROUPS[i][1] for i in self.mine if GROUPS[i][0] == 1]
        if gps:
            codes = np.stack([sample_code(ca_code(p), 1.023e6, fs, self.N) for p in gps])
            freqs = if_gps + rel
            gf = np.tile(np.arange(n_bins, dtype=np.int32), (len(gps), 1))
            self.parts.append(self._part(0, gps, codes, freqs, np.arange(len(gps)), gf))
        if glo:
            codes = sample_code(st_code(), 0.511e6, fs, self.N)[None, :]
            freqs = np.concatenate([if_glo + k * glo_step + rel for k in glo])
            gf = np.arange(len(glo) * n_bins, dtype=np.int32).reshape(len(glo), n_bins)
            self.parts.append(self._part(1, glo, codes, freqs, np.zeros(len(glo)), gf))

    def _part(self, system, ids, codes, freqs, gcode, gf):
        dev = self.device
        ctx = AcqCtx(self.fs, self.N, device=dev, max_freqs=len(freqs), max_blocks=self.n_ms,
                     max_codes=len(codes))
        ctx.set_codes(codes)
        G = len(ids)
        return dict(system=system, ids=list(ids), ctx=ctx, n_freqs=len(freqs), freqs=freqs,
                    gf=gf,
                    d_if=DevBuf(2 * self.n_ms * self.N, dev),
                    d_freqs=DevBuf.from_array(np.asarray(freqs, np.float64), dev),
                    d_gcode=DevBuf.from_array(np.asarray(gcode, np.int32), dev),
                    d_gfreq=DevBuf.from_array(np.ascontiguousarray(gf, np.int32), dev),
                    d_rows=DevBuf(G * self.n_bins * ACQ_ROW.itemsize, dev),
                    d_res=DevBuf(G * ACQ_RESULT.itemsize, dev))

    @property
    def cells(self) -> int:
        """cell-ms this rank searches per run (group x bin x code phase x ms)."""
        return len(self.mine) * self.n_bins * self.N * self.n_ms

    def load(self, if_gps: np.ndarray, if_glo: np.ndarray):
        """Interleaved int8 I,Q records of at least n_ms ms (the GPS and GLONASS front ends)."""
        need = 2 * self.n_ms * self.N
        for p in self.parts:
            rec = if_gps if p["system"] == 0 else if_glo
            p["d_if"].upload(np.ascontiguousarray(rec[:need], np.int8))

    def run(self):
        """Enqueue the search (asynchronous on each context's stream).  The two
        parts (GPS and GLONASS) run on their own streams with no join: joining
        them (both spectra first, then both correlation launches together) was
        measured slower at world 4 and 8 -- 246 workgroups from two concurrent
        launches do not all fit one round of the CUs."""
        for p in self.parts:
            G = len(p["ids"])
            p["ctx"].spectra_dev(p["d_if"].ptr, self.n_ms, p["n_freqs"], p["d_freqs"].ptr)
            p["ctx"].correlate_dev(self.n_ms, p["d_freqs"].ptr, G, self.n_bins,
                                   p["d_gcode"].ptr, p["d_gfreq"].ptr, p["d_rows"].ptr,
                                   p["d_res"].ptr, spc=self.spc, mode=ACQ_NONCOHERENT)

    def sync(self):
        for p in self.parts:
            p["ctx"].sync()

    def results(self) -> list[tuple]:
        """[(group_index, system, prn_or_fch, ACQ_RESULT record)] for this rank's groups."""
        self.sync()
        out = []
        for p in self.parts:
            res = p["d_res"].download(ACQ_RESULT, len(p["ids"]))
            for j, gid in enumerate(p["ids"]):
                gi = GROUPS.index((p["system"], gid))
                out.append((gi, p["system"], gid, res[j]))
        return sorted(out, key=lambda r: r[0])
