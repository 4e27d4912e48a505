"""oracle/acq_oracle.py -- TEST INFRASTRUCTURE ONLY.

fp64 numpy restatement of the SoftGNSS parallel code-phase acquisition, line
by line:

  GPS     POSTPROCESSING_SCILAB_RECEIVERS/GPS/L1/acquisition.sci:46-192
  GLONASS POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/acquisition.sci:46-198
  codes   GPS/L1/include/generateCAcode.sci:42-87, makeCaTable.sci:43-76,
          GLONASS/L1/include/generateSTcode.sci:35-42, makeStTable.sci:40-67

Parity status: the Scilab receivers cannot be executed here (no Scilab /
Octave / MATLAB in the image), so this restatement is pinned only
by known-answer tests (ICD first-chip octal codes, planted-signal argmax) and
by cross-agreement with the integer OSGPS oracle; it is "parity unpinned"
against a Scilab run.  Only tests/, smoke() and bench.py's cpu_baseline use it.
"""
from __future__ import annotations

import numpy as np

G2S = [5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258, 469, 470, 471,
       472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862, 145, 175, 52, 21, 237,
       235, 886, 657, 634, 762, 355, 1012, 176, 603, 130, 359, 595, 68, 386]


def generate_ca_code(prn: int) -> np.ndarray:
    """generateCAcode.sci:42-87, +-1 product-form LFSRs."""
    g2shift = G2S[prn - 1]
    g1 = np.zeros(1023)
    reg = -np.ones(10)
    for i in range(1023):
        g1[i] = reg[9]
        save = reg[2] * reg[9]
        reg[1:10] = reg[0:9].copy()
        reg[0] = save
    g2 = np.zeros(1023)
    reg = -np.ones(10)
    for i in range(1023):
        g2[i] = reg[9]
        save = reg[1] * reg[2] * reg[5] * reg[7] * reg[8] * reg[9]
        reg[1:10] = reg[0:9].copy()
        reg[0] = save
    g2 = np.concatenate([g2[1023 - g2shift:], g2[:1023 - g2shift]])
    return -(g1 * g2)


def generate_st_code() -> np.ndarray:
    """generateSTcode.sci:35-42."""
    reg = -np.ones(9)
    g3 = np.zeros(511)
    for i in range(511):
        g3[i] = reg[6]
        save = reg[4] * reg[8]
        reg[1:9] = reg[0:8].copy()
        reg[0] = save
    return -g3


def sample_code(code: np.ndarray, code_rate: float, fs: float, n: int) -> np.ndarray:
    """makeCaTable.sci:64-72 / makeStTable.sci:60-67 (1-based ceil indexing)."""
    ts = 1.0 / fs
    tc = 1.0 / code_rate
    idx = np.ceil((ts * np.arange(1, n + 1)) / tc).astype(np.int64)
    idx[-1] = len(code)
    return code[idx - 1]


def make_ca_table_row(prn: int, fs: float, n: int | None = None) -> np.ndarray:
    n = n or int(round(fs / (1.023e6 / 1023)))
    return sample_code(generate_ca_code(prn), 1.023e6, fs, n).astype(np.int8)


def make_st_table_row(fs: float, n: int | None = None) -> np.ndarray:
    n = n or int(round(fs / (0.511e6 / 511)))
    return sample_code(generate_st_code(), 0.511e6, fs, n).astype(np.int8)


def gps_bins(if_freq: float, search_band_khz: float, coh_ms: int = 1) -> np.ndarray:
    """acquisition.sci:66-67, 101-104."""
    nb = int(round(search_band_khz * 2 * coh_ms)) + 1
    k = np.arange(1, nb + 1)
    return if_freq - (search_band_khz / 2) * 1000 + (1000 / (2 * coh_ms)) * (k - 1)


def _signal(IF: np.ndarray, iq: bool) -> np.ndarray:
    x = IF.astype(np.float64)
    return x[0::2] + 1j * x[1::2] if iq else x


def power_rows(IF, fs, code, freq, n_blocks=2, iq=True) -> np.ndarray:
    """|ifft(fft(exp(i f 2 pi t) sig) conj(fft(code)))|^2 for every block."""
    N = len(code)
    sig = _signal(IF, iq)
    ts = 1.0 / fs
    phase_points = np.arange(N) * 2 * np.pi * ts            # (0:N-1)*2*%pi*ts
    sig_carr = np.exp(1j * freq * phase_points)
    cf = np.conj(np.fft.fft(code.astype(np.float64)))
    out = np.empty((n_blocks, N))
    for b in range(n_blocks):
        X = np.fft.fft(sig_carr * sig[b * N:(b + 1) * N])
        out[b] = np.abs(np.fft.ifft(X * cf)) ** 2
    return out


def _second_peak(row: np.ndarray, code_phase_1b: int, spc: int) -> float:
    """acquisition.sci:147-166, with the exclusion range as a circular open
    window (cp-spc, cp+spc); identical to the Scilab index arithmetic except
    where Scilab itself would index out of range."""
    N = len(row)
    cp = code_phase_1b - 1
    d = (np.arange(N) - cp) % N
    keep = (d >= spc) & (d <= N - spc)
    return float(row[keep].max())


def acquire(IF, fs, codes, freqs, group_freq, group_code=None, spc=16, n_blocks=2, iq=True,
            noncoherent=False, return_rows=False, coh=1):
    """Search groups (PRN/FCH) over their frequency bins.

    codes: (n_codes, N) +-1; freqs: frequency table; group_freq: (G, B) indices
    into freqs; group_code: (G,) code index per group (default arange).
    coh: settings.acqCohIntegration (GLONASS acquisition.sci:52-72, 113-135):
    blocks of coh*N samples, phase points over coh*N, the code repeated coh
    times (repmat), coh*N-point transforms; rows keep the first N powers."""
    codes = np.asarray(codes)
    group_freq = np.asarray(group_freq)
    G, B = group_freq.shape
    if group_code is None:
        group_code = np.arange(G)
    N = codes.shape[1]
    L = coh * N
    sig = _signal(IF, iq)
    ts = 1.0 / fs
    phase_points = np.arange(L) * 2 * np.pi * ts
    blocks = [sig[b * L:(b + 1) * L] for b in range(n_blocks)]
    spec = {}
    out = []
    rows_out = []
    for g in range(G):
        cf = np.conj(np.fft.fft(np.tile(codes[group_code[g]].astype(np.float64), coh)))
        results = np.zeros((B, N))
        rows = []
        for b in range(B):
            fi = int(group_freq[g, b])
            if fi not in spec:
                sc = np.exp(1j * freqs[fi] * phase_points)
                spec[fi] = [np.fft.fft(sc * blk) for blk in blocks]
            full = [np.abs(np.fft.ifft(X * cf)) ** 2 for X in spec[fi]]
            # the max picks the block over all coh*N values (:128-134), the
            # row keeps the first code period
            acq = [a[:N] for a in full]
            if coh > 1 and not noncoherent:
                chosen = 0
                for k in range(1, n_blocks):
                    if not (full[chosen].max() > full[k].max()):
                        chosen = k
                results[b] = acq[chosen]
                am = int(np.argmax(results[b]))
                rows.append(dict(peak=results[b].max(), argmax=am, block=chosen,
                                 second=_second_peak(results[b], am + 1, spc)))
                continue
            if noncoherent:
                results[b] = np.sum(acq, axis=0)
                chosen = 0
            else:
                # acquisition.sci:126-132 (n_blocks == 2); generalised: a later
                # block replaces the kept one unless the kept max is larger
                chosen = 0
                for k in range(1, n_blocks):
                    if not (acq[chosen].max() > acq[k].max()):
                        chosen = k
                results[b] = acq[chosen]
            am = int(np.argmax(results[b]))
            rows.append(dict(peak=results[b].max(), argmax=am, block=chosen,
                             second=_second_peak(results[b], am + 1, spc)))
        row_max = results.max(axis=1)
        peak = row_max.max()
        bin_idx = int(np.argmax(row_max))                   # max(max(results,'c'))
        code_phase = int(np.argmax(results.max(axis=0))) + 1  # max(max(results,'r'))
        second = _second_peak(results[bin_idx], code_phase, spc)
        out.append(dict(peak=peak, second=second, metric=peak / second, bin=bin_idx,
                        code_phase=code_phase, carr_freq=float(freqs[group_freq[g, bin_idx]])))
        rows_out.append(rows)
    return (out, rows_out) if return_rows else out


def acquire_batched(IF, fs, codes, freqs, group_freq, group_code=None, spc=16, n_blocks=2,
                    iq=True, workers=1):
    """Same fp64 algorithm as acquire(), batched over bins with scipy's
    multithreaded pocketfft.  Used as bench.py's CPU baseline only."""
    import scipy.fft as sfft
    codes = np.asarray(codes)
    group_freq = np.asarray(group_freq)
    G, B = group_freq.shape
    if group_code is None:
        group_code = np.arange(G)
    N = codes.shape[1]
    sig = _signal(IF, iq)[:n_blocks * N].reshape(n_blocks, N)
    phase_points = np.arange(N) * 2 * np.pi * (1.0 / fs)
    fidx = np.unique(group_freq)
    carr = np.exp(1j * np.asarray(freqs)[fidx][:, None] * phase_points[None, :])
    spec = sfft.fft(carr[:, None, :] * sig[None, :, :], axis=-1, workers=workers)
    row_of = {int(f): i for i, f in enumerate(fidx)}
    out = []
    for g in range(G):
        cf = np.conj(sfft.fft(codes[group_code[g]].astype(np.float64), workers=workers))
        X = spec[[row_of[int(f)] for f in group_freq[g]]]          # (B, blocks, N)
        P = np.abs(sfft.ifft(X * cf[None, None, :], axis=-1, workers=workers)) ** 2
        mx = P.max(axis=-1)                                          # (B, blocks)
        chosen = np.zeros(B, np.int64)
        for k in range(1, n_blocks):
            repl = ~(mx[np.arange(B), chosen] > mx[:, k])
            chosen[repl] = k
        results = P[np.arange(B), chosen]
        row_max = results.max(axis=1)
        bin_idx = int(np.argmax(row_max))
        code_phase = int(np.argmax(results.max(axis=0))) + 1
        second = _second_peak(results[bin_idx], code_phase, spc)
        out.append(dict(peak=row_max.max(), second=second, metric=row_max.max() / second,
                        bin=bin_idx, code_phase=code_phase))
    return out
