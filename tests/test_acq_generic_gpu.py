"""GPU parity of the generic-N fp64 acquisition (csrc/acq64.hip): any
samplesPerCode = round(fs / (codeFreqBasis / codeLength)) (acquisition.sci:47-48)
without a compiled prime-factor plan, e.g. fs = 5 MHz (N = 5000) or the classic
SoftGNSS front end at 38.192 MHz (N = 38192).

Held to the same bar as the compiled plans (tests/test_acq_gpu.py check_rows,
fp64 class): powers, peaks, second peaks and metrics within 1e-6 relative of the
fp64 oracle (oracle/acq_oracle.py; observed ~1e-13), code phase and bin exact.
Two engines: the mixed-radix Stockham plan (N a product of radices <= 31:
5000 = 8 x 5^4, 38192 = 16 x 7 x 11 x 31; the default; where a four-step plan is
compiled, 38192 = 112 x 341 and 16368 = 48 x 341, its two LDS passes replace the
four global ones, GNSSCORR_ACQ_MIX4=0 keeps the passes) and Bluestein's chirp-z
(prime factors above 31, or GNSSCORR_ACQ_BLUESTEIN=1); both are held to the
oracle and to each other.  The generic engine also runs at N = 16368
(GNSSCORR_ACQ_GENERIC=1) against the compiled 16 x 33 x 31 plan.
"""
import numpy as np
import pytest

import acq_oracle as A
from test_acq_gpu import check_rows

pytestmark = pytest.mark.gpu


def _scene(gpu, fs, n_ms, seed):
    sigs = [dict(system=0, prn=6, code_phase=211.7, doppler=-1750.0, cn0=47.0),
            dict(system=0, prn=19, code_phase=804.2, doppler=2250.0, cn0=49.0)]
    return gpu.ifgen(n_ms * int(round(fs / 1000.0)), sigs, fs=fs, seed=seed)


@pytest.mark.parametrize("engine", ["mixed", "bluestein"])
@pytest.mark.parametrize("fs", [5.0e6, 38.192e6, 4.111e6])
def test_power_row_generic(gpu, fs, engine, monkeypatch):
    """4.111 MHz: N = 4111 is prime, Bluestein either way."""
    monkeypatch.setenv("GNSSCORR_ACQ_BLUESTEIN", "1" if engine == "bluestein" else "0")
    n = int(round(fs / 1000.0))
    ctx = gpu.AcqCtx(fs, n, max_freqs=4, max_blocks=2, max_codes=2)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (19, 6)])
    assert codes.shape[1] == n
    ctx.set_codes(codes)
    IF = _scene(gpu, fs, 2, 0x5EED0020)
    for code, freq, blk in [(0, 2.42e6 + 2250.0, 0), (1, 2.42e6 - 1750.0, 1)]:
        got = ctx.power_row(IF, 2, blk, freq, code)
        ref = A.power_rows(IF, fs, codes[code], freq)[blk]
        err = np.abs(got - ref).max() / ref.max()
        print(f"[generic power row N={n}] code {code}: {err:.3e}")
        assert err < 1e-9
        assert np.argmax(got) == np.argmax(ref)


@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_search_5000(gpu, mode):
    fs, n = 5.0e6, 5000
    nb = 2 if mode == "best" else 4
    ctx = gpu.AcqCtx(fs, n, max_freqs=64, max_blocks=nb, max_codes=4)
    prns = [6, 11, 19]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    ctx.set_codes(codes)
    IF = _scene(gpu, fs, nb, 0x5EED0021)
    freqs = A.gps_bins(2.42e6, 14, 1)
    gf = np.tile(np.arange(len(freqs)), (3, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    res, rows = ctx.search(IF, nb, freqs, np.arange(3), gf, spc=5, mode=m)
    ref, ref_rows = A.acquire(IF, fs, codes, freqs, gf, spc=5, n_blocks=nb,
                              noncoherent=mode == "noncoherent", return_rows=True)
    if mode == "noncoherent":          # the non-coherent rows carry no block choice
        for rr in ref_rows:
            for r in rr:
                r["block"] = -1
    check_rows(res, rows, ref, ref_rows, True, label=f"generic-5000-{mode}")
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5


def test_generic_packed_equals_int8(gpu):
    fs, n = 5.0e6, 5000
    IF = _scene(gpu, fs, 2, 0x5EED0022)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (6, 19)])
    freqs = A.gps_bins(2.42e6, 6, 1)
    out = []
    for packed in (False, True):
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=2, max_codes=2)
        ctx.set_codes(codes)
        out.append(ctx.search(gpu.pack2(IF) if packed else IF, 2, freqs, np.arange(2),
                              np.tile(np.arange(len(freqs)), (2, 1)), spc=5,
                              iq=gpu.iq_flags(True, packed)))
    assert out[0][0].tobytes() == out[1][0].tobytes()
    assert out[0][1].tobytes() == out[1][1].tobytes()


def test_generic_engine_at_16368_matches_compiled_plan(gpu, monkeypatch):
    fs, n = 16.368e6, 16368
    IF = gpu.ifgen(2 * n, [dict(system=0, prn=9, code_phase=500.5, doppler=1500.0, cn0=47.0)],
                   fs=fs, seed=0x5EED0023)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (9, 23)])
    freqs = 2.42e6 + 500.0 * np.arange(-6, 7)
    gf = np.tile(np.arange(len(freqs)), (2, 1))
    out = []
    for generic in ("0", "1"):
        monkeypatch.setenv("GNSSCORR_ACQ_GENERIC", generic)
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=2, max_codes=2)
        ctx.set_codes(codes)
        out.append(ctx.search(IF, 2, freqs, np.arange(2), gf, spc=16))
    (r0, w0), (r1, w1) = out
    assert (r0["code_phase"] == r1["code_phase"]).all() and (r0["bin"] == r1["bin"]).all()
    assert (w0["argmax"] == w1["argmax"]).all()
    rel = np.abs(w0["peak"] - w1["peak"]) / w0["peak"]
    print(f"[generic vs PFA at 16368] max peak rel diff {rel.max():.3e}")
    assert rel.max() < 1e-9
    assert np.allclose(r0["metric"], r1["metric"], rtol=1e-9)


@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_search_38192_mixed_radix(gpu, mode):
    """The classic SoftGNSS front end (N = 38192 = 16 x 7 x 11 x 31, the mixed-radix
    plan) against the oracle: 3 PRNs x 9 bins."""
    fs, n = 38.192e6, 38192
    nb = 2
    ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=nb, max_codes=3)
    prns = [6, 11, 19]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    ctx.set_codes(codes)
    IF = _scene(gpu, fs, nb, 0x5EED0024)
    freqs = 2.42e6 + 500.0 * np.arange(-4, 5)
    gf = np.tile(np.arange(len(freqs)), (3, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    res, rows = ctx.search(IF, nb, freqs, np.arange(3), gf, spc=37, mode=m)
    ref, ref_rows = A.acquire(IF, fs, codes, freqs, gf, spc=37, n_blocks=nb,
                              noncoherent=mode == "noncoherent", return_rows=True)
    if mode == "noncoherent":
        for rr in ref_rows:
            for r in rr:
                r["block"] = -1
    check_rows(res, rows, ref, ref_rows, True, label=f"mixed-38192-{mode}")
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5


@pytest.mark.parametrize("fs", [5.0e6, 38.192e6])
def test_mixed_radix_equals_bluestein(gpu, fs, monkeypatch):
    """The two generic engines on one search: decisions identical, powers within
    1e-9 relative of each other (both are fp64 DFTs of the same rows)."""
    n = int(round(fs / 1000.0))
    IF = _scene(gpu, fs, 2, 0x5EED0025)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (6, 19, 25)])
    freqs = 2.42e6 + 500.0 * np.arange(-6, 7)
    gf = np.tile(np.arange(len(freqs)), (3, 1))
    out = []
    for bl in ("0", "1"):
        monkeypatch.setenv("GNSSCORR_ACQ_BLUESTEIN", bl)
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=2, max_codes=3)
        ctx.set_codes(codes)
        out.append(ctx.search(IF, 2, freqs, np.arange(3), gf, spc=int(round(fs / 1.023e6))))
    (r0, w0), (r1, w1) = out
    assert (r0["code_phase"] == r1["code_phase"]).all() and (r0["bin"] == r1["bin"]).all()
    assert (w0["argmax"] == w1["argmax"]).all() and (w0["block"] == w1["block"]).all()
    rel = np.abs(w0["peak"] - w1["peak"]) / w0["peak"]
    rel2 = np.abs(w0["second"] - w1["second"]) / w0["second"]
    print(f"[mixed vs bluestein N={n}] peak {rel.max():.3e} second {rel2.max():.3e}")
    assert rel.max() < 1e-9 and rel2.max() < 1e-9


@pytest.mark.parametrize("mode", ["best", "noncoherent"])
@pytest.mark.parametrize("fs,generic", [(38.192e6, "0"), (16.368e6, "1")])
def test_four_step_equals_mixed_radix_passes(gpu, fs, generic, mode, monkeypatch):
    """The four-step plan (m4_cols2 / m4_rows2: 112 x 341 at 38.192 Msps, 48 x 341 at
    16.368 Msps on the generic engine) against the four mixed-radix passes
    (GNSSCORR_ACQ_MIX4=0) on one search: decisions identical, peaks and second
    peaks within 1e-9 relative (both fp64 DFTs of the same rows)."""
    monkeypatch.setenv("GNSSCORR_ACQ_GENERIC", generic)
    n = int(round(fs / 1000.0))
    IF = _scene(gpu, fs, 2, 0x5EED0026)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (6, 19, 25)])
    freqs = 2.42e6 + 500.0 * np.arange(-6, 7)
    gf = np.tile(np.arange(len(freqs)), (3, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    out = []
    for m4 in ("1", "0"):
        monkeypatch.setenv("GNSSCORR_ACQ_MIX4", m4)
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=2, max_codes=3)
        ctx.set_codes(codes)
        out.append(ctx.search(IF, 2, freqs, np.arange(3), gf, spc=int(round(fs / 1.023e6)), mode=m))
    (r0, w0), (r1, w1) = out
    assert (r0["code_phase"] == r1["code_phase"]).all() and (r0["bin"] == r1["bin"]).all()
    assert (w0["argmax"] == w1["argmax"]).all() and (w0["block"] == w1["block"]).all()
    rel = np.abs(w0["peak"] - w1["peak"]) / w0["peak"]
    rel2 = np.abs(w0["second"] - w1["second"]) / w0["second"]
    print(f"[four-step vs passes N={n} {mode}] peak {rel.max():.3e} second {rel2.max():.3e}")
    assert rel.max() < 1e-9 and rel2.max() < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("fs,generic", [(38.192e6, "0"), (16.368e6, "1")])
@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_four_step_fused_statistics_equal_stats_pass(gpu, fs, generic, mode, monkeypatch):
    """The row statistics fused into the four-step plan's last m4_rows2 (per-column
    top-2, then m4_stats_kernel over the N1 columns) against the separate one-pass
    statistics kernel over the stored power rows (GNSSCORR_ACQ_M4STATS=0): the same
    power values feed both, so every peak, second peak, argmax and block is equal
    bit for bit."""
    monkeypatch.setenv("GNSSCORR_ACQ_GENERIC", generic)
    n = int(round(fs / 1000.0))
    IF = _scene(gpu, fs, 2, 0x5EED0027)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (3, 11, 30)])
    freqs = 2.42e6 + 500.0 * np.arange(-6, 7)
    gf = np.tile(np.arange(len(freqs)), (3, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    out = []
    for st in ("1", "0"):
        monkeypatch.setenv("GNSSCORR_ACQ_M4STATS", st)
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=2, max_codes=3)
        ctx.set_codes(codes)
        out.append(ctx.search(IF, 2, freqs, np.arange(3), gf, spc=int(round(fs / 1.023e6)), mode=m))
    (r0, w0), (r1, w1) = out
    for k in ("code_phase", "bin"):
        assert (r0[k] == r1[k]).all(), k
    for k in ("peak", "second", "argmax", "block"):
        assert (w0[k] == w1[k]).all(), k


@pytest.mark.parametrize("m4stats", ["1", "0"])
@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_generic_multi_chunk_16368(gpu, mode, m4stats, monkeypatch):
    """The chunk loop on the other four-step plan (48 x 341: m4_cols2<3, 16>): the
    generic engine forced at 16.368 Msps with 1 MiB of Y per chunk (3 rows of 48 x 352
    complex), so the carried statistics and u0 > 0 run with A = 3 as well."""
    monkeypatch.setenv("GNSSCORR_ACQ_GENERIC", "1")
    monkeypatch.setenv("GNSSCORR_ACQ_GCHUNK_MB", "1")
    monkeypatch.setenv("GNSSCORR_ACQ_M4STATS", m4stats)
    fs, n, nb = 16.368e6, 16368, 2
    ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=nb, max_codes=4)
    prns = [6, 11, 19, 25]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    ctx.set_codes(codes)
    IF = _scene(gpu, fs, nb, 0x5EED0029)
    freqs = 2.42e6 + 500.0 * np.arange(-4, 5)
    gf = np.tile(np.arange(len(freqs)), (4, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    res, rows = ctx.search(IF, nb, freqs, np.arange(4), gf, spc=16, mode=m)
    ref, ref_rows = A.acquire(IF, fs, codes, freqs, gf, spc=16, n_blocks=nb,
                              noncoherent=mode == "noncoherent", return_rows=True)
    if mode == "noncoherent":
        for rr in ref_rows:
            for r in rr:
                r["block"] = -1
    check_rows(res, rows, ref, ref_rows, True, label=f"chunked-16368-{mode}-m4stats{m4stats}")
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5


@pytest.mark.parametrize("m4stats", ["1", "0"])
@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_generic_multi_chunk_38192(gpu, mode, m4stats, monkeypatch):
    """The generic engine's chunk loop: GNSSCORR_ACQ_GCHUNK_MB=2 gives
    3 rows per chunk at N = 38192, so the 4-code spectra take 2 chunks, the 4 class rows
    2, and the 4 x 9 (x 2 blocks) units 12-24 chunks: every chunk after the first runs
    with u0 > 0 in MixCorr, m4_launch and the fused statistics (fused on: carried by
    the next chunk's m4_cols2, the last chunk's by m4_stats_kernel) or g_stats1_kernel
    (off).  Against the fp64 oracle (SCI/GPS/L1/acquisition.sci:98-169)."""
    monkeypatch.setenv("GNSSCORR_ACQ_GCHUNK_MB", "2")
    monkeypatch.setenv("GNSSCORR_ACQ_M4STATS", m4stats)
    fs, n, nb = 38.192e6, 38192, 2
    ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=nb, max_codes=4)
    prns = [6, 11, 19, 25]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    ctx.set_codes(codes)
    IF = _scene(gpu, fs, nb, 0x5EED0028)
    freqs = 2.42e6 + 500.0 * np.arange(-4, 5)
    gf = np.tile(np.arange(len(freqs)), (4, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    res, rows = ctx.search(IF, nb, freqs, np.arange(4), gf, spc=37, mode=m)
    ref, ref_rows = A.acquire(IF, fs, codes, freqs, gf, spc=37, n_blocks=nb,
                              noncoherent=mode == "noncoherent", return_rows=True)
    if mode == "noncoherent":
        for rr in ref_rows:
            for r in rr:
                r["block"] = -1
    check_rows(res, rows, ref, ref_rows, True, label=f"chunked-38192-{mode}-m4stats{m4stats}")
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5


@pytest.mark.parametrize("engine", ["four_step", "passes", "bluestein"])
def test_second_peak_window_across_the_wrap(gpu, engine, monkeypatch):
    """the one-pass statistics' thread t holds samples t and
    t + 1024 q, only N - 1024 q = 304 apart across the wrap at N = 38192.  Two copies of
    PRN 6 put the correlation peak at sample 101 and a weaker one at 37989 (thread 101's
    last sample, 304 before it circularly).  With spc = 400 the weaker peak lies inside
    the open window (argmax - spc, argmax + spc), so the second peak must come from
    outside it (acquisition.sci:150-165); a one-pass thread runner-up would report the
    weaker copy.  Scene checked on the host: oracle second 5.5e6, weaker peak 8.7e7."""
    monkeypatch.setenv("GNSSCORR_ACQ_BLUESTEIN", "1" if engine == "bluestein" else "0")
    monkeypatch.setenv("GNSSCORR_ACQ_MIX4", "0" if engine == "passes" else "1")
    fs, n, nb, spc = 38.192e6, 38192, 2, 400
    spc_n = n / 1023.0
    p1, p2 = 100, 100 + 37888
    IF = gpu.ifgen(nb * n, [dict(system=0, prn=6, code_phase=(n - p1) / spc_n, doppler=500.0,
                                 cn0=60.0),
                            dict(system=0, prn=6, code_phase=(n - p2) / spc_n, doppler=500.0,
                                 cn0=56.0)], fs=fs, seed=7)
    codes = np.stack([A.make_ca_table_row(6, fs)])
    freqs = 2.42e6 + 500.0 * np.arange(-1, 2)
    gf = np.arange(3)[None, :]
    ctx = gpu.AcqCtx(fs, n, max_freqs=4, max_blocks=nb, max_codes=1)
    ctx.set_codes(codes)
    res, rows = ctx.search(IF, nb, freqs, np.arange(1), gf, spc=spc)
    ref, ref_rows = A.acquire(IF, fs, codes, freqs, gf, spc=spc, n_blocks=nb, return_rows=True)
    r = ref_rows[0][2]
    assert r["argmax"] == p1 + 1 and r["second"] < 0.1 * r["peak"]   # the trap is set
    check_rows(res, rows, ref, ref_rows, True, label=f"wrap-window-{engine}")


@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_generic_bench_scale_38192(gpu, mode):
    """The bench's generic-rate search at full scale (bench.py run_acq_generic): 32 PRNs
    x 41 bins x 2 blocks at 38.192 Msps with the default work buffer, i.e. the chunking
    the bench runs (best: 2 624 units in 14 equal chunks of 188 on two chunk lanes, each
    chunk's statistics carried by its lane's next column pass; non-coherent: 1 312 rows in
    8 chunks), every row's statistics against the fp64 oracle
    (SCI/GPS/L1/acquisition.sci:98-169)."""
    fs, n, nb = 38.192e6, 38192, 2
    rng = np.random.default_rng(300)
    planted = rng.choice(np.arange(1, 33), 8, replace=False)
    sigs = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
                 doppler=float(rng.uniform(-5000, 5000)), cn0=49.0, data_bits=1) for p in planted]
    IF = gpu.ifgen(nb * n, sigs, fs=fs, seed=0x5EED0030)
    ctx = gpu.AcqCtx(fs, n, max_freqs=41, max_blocks=nb, max_codes=32)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in range(1, 33)])
    ctx.set_codes(codes)
    freqs = 2.42e6 - 10000.0 + 500.0 * np.arange(41)
    gf = np.tile(np.arange(41), (32, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    res, rows = ctx.search(IF, nb, freqs, np.arange(32), gf, spc=37, mode=m)
    ref, ref_rows = A.acquire(IF, fs, codes, freqs, gf, spc=37, n_blocks=nb,
                              noncoherent=mode == "noncoherent", return_rows=True)
    if mode == "noncoherent":
        for rr in ref_rows:
            for r in rr:
                r["block"] = -1
    worst = check_rows(res, rows, ref, ref_rows, True, label=f"bench-scale-38192-{mode}")
    print(f"[generic bench scale {mode}] worst rel {worst:.3e}")
    assert all(res[p - 1]["metric"] > 2.5 for p in planted)


@pytest.mark.parametrize("m4stats", ["1", "0"])
@pytest.mark.parametrize("mode", ["best", "noncoherent"])
def test_two_lanes_equal_one_lane(gpu, mode, m4stats, monkeypatch):
    """The four-step plan's two chunk lanes (odd chunks on a second stream with their own
    Y, power rows and column top-2) give byte-identical rows and results to one lane
    (GNSSCORR_ACQ_M4LANES=1), over many chunks (2 MiB: 6 rows per lane chunk)."""
    fs, n, nb = 38.192e6, 38192, 2
    prns = [6, 11, 19, 25]
    codes = np.stack([A.make_ca_table_row(p, fs) for p in prns])
    IF = _scene(gpu, fs, nb, 0x5EED002A)
    freqs = 2.42e6 + 500.0 * np.arange(-6, 7)
    gf = np.tile(np.arange(len(freqs)), (4, 1))
    m = gpu.ACQ_NONCOHERENT if mode == "noncoherent" else gpu.ACQ_BEST_OF_BLOCKS
    monkeypatch.setenv("GNSSCORR_ACQ_GCHUNK_MB", "4")
    monkeypatch.setenv("GNSSCORR_ACQ_M4STATS", m4stats)
    out = {}
    for lanes in ("2", "1"):
        monkeypatch.setenv("GNSSCORR_ACQ_M4LANES", lanes)
        ctx = gpu.AcqCtx(fs, n, max_freqs=16, max_blocks=nb, max_codes=4)
        ctx.set_codes(codes)
        out[lanes] = ctx.search(IF, nb, freqs, np.arange(4), gf, spc=37, mode=m)
    (r2, w2), (r1, w1) = out["2"], out["1"]
    assert r2.tobytes() == r1.tobytes()
    assert w2.tobytes() == w1.tobytes()
    assert r1[0]["metric"] > 2.5 and r1[2]["metric"] > 2.5
