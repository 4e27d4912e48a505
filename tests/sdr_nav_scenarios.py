"""Synthetic prompt-correlation streams for the GPS-SDR Channel (bit lock, frame
sync, parity, C/N0, loops): ICD-GPS-200 navigation words with their parity
(the inverse of Channel::ParityCheck, channel.cpp:784-812), subframes 1..5
with preamble / HOW / zero t bits as FrameSync and ValidFrameFormat
(channel.cpp:731-904) expect, 50 bps BPSK on 1-ms E/P/L correlations.

Test infrastructure only (tests/ and tests/golden/make_sdr_chan_golden.py).
"""
from __future__ import annotations

import numpy as np

PREAMBLE = 0x8B

# ICD-GPS-200 table 20-XIV: data bits d1..d24 taking part in parity bits D25..D30
_PAR = [
    (29, [1, 2, 3, 5, 6, 10, 11, 12, 13, 14, 17, 18, 20, 23]),
    (30, [2, 3, 4, 6, 7, 11, 12, 13, 14, 15, 18, 19, 21, 24]),
    (29, [1, 3, 4, 5, 7, 8, 12, 13, 14, 15, 16, 19, 20, 22]),
    (30, [2, 4, 5, 6, 8, 9, 13, 14, 15, 16, 17, 20, 21, 23]),
    (30, [1, 3, 5, 6, 7, 9, 10, 14, 15, 16, 17, 18, 21, 22, 24]),
    (29, [3, 5, 6, 8, 9, 10, 11, 13, 15, 19, 22, 23, 24]),
]


def encode_word(d24: int, prev: int) -> int:
    """30-bit transmitted word (D1 = bit 29) from 24 source data bits, given the
    previous transmitted word (its D29*, D30* = bits 1, 0)."""
    d29s, d30s = (prev >> 1) & 1, prev & 1
    d = [(d24 >> (24 - i)) & 1 for i in range(1, 25)]         # d[0] = d1
    out = 0
    for i in range(24):
        out = (out << 1) | (d[i] ^ d30s)
    for star, idx in _PAR:
        p = d29s if star == 29 else d30s
        for i in idx:
            p ^= d[i - 1]
        out = (out << 1) | p
    return out


def parity_ok(word: int) -> bool:
    """Channel::ParityCheck (channel.cpp:784-812) on a word whose data bits are
    already un-inverted (bits 31-30 = D29*, D30* of the previous word)."""
    def rotl(x, n):
        return ((x << n) ^ (x >> (32 - n))) & 0xFFFFFFFF
    w = word & 0xFFFFFFFF
    t = (w & 0xFBFFBF00) ^ (rotl(w, 1) & 0x07FFBF01) ^ (rotl(w, 2) & 0xFC0F8100) ^ \
        (rotl(w, 3) & 0xF81FFE02) ^ (rotl(w, 4) & 0xFC00000E) ^ (rotl(w, 5) & 0x07F00001) ^ \
        (rotl(w, 6) & 0x00003000)
    par = (t ^ rotl(t, 6) ^ rotl(t, 12) ^ rotl(t, 18) ^ rotl(t, 24)) & 0x3F
    return par == (w & 0x3F)


def subframe_bits(sid: int, tow: int, rng: np.random.Generator, prev: int = 0) -> tuple:
    """300 transmitted bits of subframe sid (1..5) with TOW count tow; returns
    (bits uint8[300], last transmitted word)."""
    words = []
    tlm = (PREAMBLE << 16) | int(rng.integers(0, 1 << 14)) << 2
    w = encode_word(tlm, prev)
    words.append(w)
    prev = w
    # HOW: 17-bit TOW, 2 flag bits, 3-bit subframe ID, 2 t bits chosen so that
    # D29 = D30 = 0 (FrameSync / ValidFrameFormat "zero bits")
    for t in range(4):
        how = (tow & 0x1FFFF) << 7 | (sid & 7) << 2 | t
        cand = encode_word(how, prev)
        if cand & 3 == 0:
            break
    words.append(cand)
    prev = cand
    for k in range(8):
        d = int(rng.integers(0, 1 << 24))
        if k == 7:   # word 10: t bits make D29 = D30 = 0 (the next TLM's D29*, D30*)
            for t in range(4):
                w = encode_word((d & ~3) | t, prev)
                if w & 3 == 0:
                    break
        else:
            w = encode_word(d, prev)
        words.append(w)
        prev = w
    bits = np.array([(w >> (29 - i)) & 1 for w in words for i in range(30)], np.uint8)
    return bits, prev


def nav_bits(n_subframes: int, seed: int, tow0: int = 1000, sid0: int = 1) -> np.ndarray:
    rng = np.random.default_rng(seed)
    out, prev = [], 0
    for k in range(n_subframes):
        b, prev = subframe_bits((sid0 - 1 + k) % 5 + 1, tow0 + k, rng, prev)
        out.append(b)
    return np.concatenate(out)


def correlations(n_ms: int, bits: np.ndarray, bit_offset_ms: int, amp: float, noise: float,
                 seed: int, q_bias: float = 0.0, el_frac: float = 0.5,
                 fade_after_ms: int = -1) -> np.ndarray:
    """[n_ms, 6] int32 Correlation_S rows (I_E, I_P, I_L, Q_E, Q_P, Q_L) of a
    50 bps BPSK signal: bit k covers ms [bit_offset + 20k, bit_offset + 20k + 20).
    fade_after_ms >= 0 drops the signal to noise from that ms on (loss of lock)."""
    rng = np.random.default_rng(seed)
    ms = np.arange(n_ms)
    k = np.clip((ms - bit_offset_ms) // 20, 0, len(bits) - 1)
    s = (2.0 * bits[k].astype(np.float64) - 1.0) * amp
    if fade_after_ms >= 0:
        s[fade_after_ms:] = 0.0
    out = np.empty((n_ms, 6), np.int64)
    g = rng.standard_normal((n_ms, 6)) * noise
    out[:, 0] = np.rint(el_frac * s + g[:, 0])
    out[:, 1] = np.rint(s + g[:, 1])
    out[:, 2] = np.rint(el_frac * s + g[:, 2])
    out[:, 3] = np.rint(q_bias * el_frac * s + g[:, 3])
    out[:, 4] = np.rint(q_bias * s + g[:, 4])
    out[:, 5] = np.rint(q_bias * el_frac * s + g[:, 5])
    return out.astype(np.int32)


# scenario table: (sv, doppler, corr_len, bit_offset_ms, amp, noise, q_bias, fade_after_ms)
SCENARIOS = [
    (0, 1250, 1, 7, 4000.0, 900.0, 0.02, -1),     # strong: bit lock, frame sync, subframes
    (4, -3000, 1, 13, 2600.0, 1300.0, -0.05, -1),  # weaker: C/N0 below 37 -> 20-ms dumps
    (11, 400, 20, 0, 3500.0, 700.0, 0.0, -1),     # started with 20-ms integration
    (20, 7000, 1, 19, 4000.0, 800.0, 0.1, 9000),  # fades: P_avg < 8e4 -> Kill
]
