"""GPU: BASELINE config 5 -- full-sky (32 GPS PRN + 14 GLONASS FCH) x 41 bins,
10 ms non-coherent, groups sharded over ranks (gnsscorr/fullsky.py).

Checks: (1) planted groups vs the fp64 acquisition.sci oracle (non-coherent
sum of |ifft|^2 over 10 blocks, oracle/acq_oracle.py; fp64, so the
north_star 1e-6 relative tolerance and exact decisions); (2) sharding is exact: the union of the rank-0 and
rank-1 shards of a 2-way split equals the unsharded search bit for bit (each
group's search is independent).
"""
import numpy as np
import pytest

import acq_oracle as A

pytestmark = pytest.mark.gpu
FS = 16.368e6
N = 16368


@pytest.fixture(scope="module")
def scene(gpu):
    rng = np.random.default_rng(55)
    gps = [(5, 100.0, 1500.0), (13, 700.5, -3200.0), (24, 50.0, 4100.0), (31, 999.0, -800.0)]
    glo = [(-6, 20.0, 2500.0), (0, 300.0, -1200.0), (5, 480.0, 700.0)]
    sg = [dict(system=0, prn=p, code_phase=c, doppler=d, cn0=41.0, data_bits=1) for p, c, d in gps]
    sl = [dict(system=1, fch=k, code_phase=c, doppler=d, cn0=43.0, data_bits=1)
          for k, c, d in glo]
    if_gps = gpu.ifgen(10 * N, sg, fs=FS, seed=int(rng.integers(1 << 30)))
    if_glo = gpu.ifgen(10 * N, sl, fs=FS, if_glo=1.0e6, seed=int(rng.integers(1 << 30)))
    return dict(gps=gps, glo=glo, if_gps=if_gps, if_glo=if_glo)


def _run(gpu, scene, world, rank):
    from gnsscorr.fullsky import FullSky
    fs = FullSky(FS, 10, 41, rank=rank, world=world)
    fs.load(scene["if_gps"], scene["if_glo"])
    fs.run()
    return fs.results()


def test_fullsky_planted_vs_oracle(gpu, scene):
    from gnsscorr.fullsky import merge
    res = merge([_run(gpu, scene, 1, 0)])
    assert len(res) == 46
    freqs_rel = 500.0 * (np.arange(41) - 20)
    for prn, cp, dop in scene["gps"]:
        r = res[prn - 1][3]
        code = A.make_ca_table_row(prn, FS)[None, :]
        ref = A.acquire(scene["if_gps"], FS, code, 2.42e6 + freqs_rel, np.arange(41)[None, :],
                        n_blocks=10, noncoherent=True)[0]
        assert abs(r["peak"] - ref["peak"]) <= 1e-6 * ref["peak"], prn
        assert abs(r["metric"] - ref["metric"]) <= 1e-6 * ref["metric"], prn
        assert r["bin"] == ref["bin"] and r["code_phase"] == ref["code_phase"], prn
        assert r["metric"] > 2.5
        assert abs(r["carr_freq"] - (2.42e6 + dop)) <= 250.0
    st = A.make_st_table_row(FS)[None, :]
    for k, cp, dop in scene["glo"]:
        r = res[32 + k + 7][3]
        f = 1.0e6 + k * 0.5625e6 + freqs_rel
        ref = A.acquire(scene["if_glo"], FS, st, f, np.arange(41)[None, :], n_blocks=10,
                        noncoherent=True)[0]
        assert abs(r["peak"] - ref["peak"]) <= 1e-6 * ref["peak"], k
        assert abs(r["metric"] - ref["metric"]) <= 1e-6 * ref["metric"], k
        assert r["bin"] == ref["bin"] and r["code_phase"] == ref["code_phase"], k
        assert r["metric"] > 2.5


def test_fullsky_sharding_is_exact(gpu, scene):
    from gnsscorr.fullsky import merge
    one = merge([_run(gpu, scene, 1, 0)])
    two = merge([_run(gpu, scene, 2, 0), _run(gpu, scene, 2, 1)])
    three = merge([_run(gpu, scene, 3, r) for r in range(3)])
    eight = merge([_run(gpu, scene, 8, r) for r in range(8)])
    for a, b, c, d in zip(one, two, three, eight):
        assert a[:3] == b[:3] == c[:3] == d[:3]
        assert a[3].tobytes() == b[3].tobytes() == c[3].tobytes() == d[3].tobytes(), a[:3]


def test_group_records_equal_separate_searches(gpu):
    """gnsscorr_acq_set_group_records: groups of two IF records in one launch give
    the same bytes as each record searched alone (two PRNs on record 0, one on 1)."""
    fs, n = FS, N
    s0 = [dict(system=0, prn=3, code_phase=210.0, doppler=1200.0, cn0=45.0)]
    s1 = [dict(system=0, prn=17, code_phase=640.5, doppler=-2600.0, cn0=45.0)]
    r0 = gpu.ifgen(4 * n, s0, fs=fs, seed=0x5EED0051)
    r1 = gpu.ifgen(4 * n, s1, fs=fs, seed=0x5EED0052)
    codes = np.stack([A.make_ca_table_row(p, fs) for p in (3, 9, 17)])
    freqs = 2.42e6 + 500.0 * np.arange(-8, 9)
    nb = len(freqs)
    gf = np.tile(np.arange(nb, dtype=np.int32), (3, 1))
    for mode in (gpu.ACQ_BEST_OF_BLOCKS, gpu.ACQ_NONCOHERENT):
        both = gpu.AcqCtx(fs, n, max_freqs=nb, max_blocks=8, max_codes=3)
        both.set_codes(codes)
        both.set_records(2)
        d_rec = gpu.DevBuf.from_array(np.array([0, 0, 1], np.int32))
        both.set_group_records(d_rec)
        res, rows = both.search(np.concatenate([r0, r1]), 4, freqs, [0, 1, 2], gf, mode=mode)
        for g, rec in ((0, r0), (1, r0), (2, r1)):
            one = gpu.AcqCtx(fs, n, max_freqs=nb, max_blocks=4, max_codes=3)
            one.set_codes(codes)
            ra, wa = one.search(rec, 4, freqs, [g], gf[:1], mode=mode)
            assert res[g].tobytes() == ra[0].tobytes(), (mode, g)
            assert rows[g].tobytes() == wa[0].tobytes(), (mode, g)
    assert res[0]["metric"] > 2.5 and res[2]["metric"] > 2.5
