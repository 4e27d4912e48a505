"""GPU: tracking channels sharded over ranks (gnsscorr/trackshard.py).

4 receivers x 12 GP2021 channels, 6 consecutive 1-ms calls.  The same channel
set is run unsharded (world 1) and as world-2 / world-3 shards (separate
contexts on the one local GPU standing in for the ranks); merged by global
channel index, every call's TRACK_RESULT must equal the unsharded run bit for
bit -- channels are independent (correlator.c:149-316), so sharding cannot
change a single accumulator.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FS, NS, RX, CH, CALLS = 16.368e6, 16368, 4, 12, 6


def _cmds(gc, rng):
    c = np.zeros(RX * CH, gc.NCO_CMD)
    c["prn"] = rng.integers(1, 33, RX * CH)
    c["stream"] = np.repeat(np.arange(RX), CH)
    c["carrier_incr"] = 635008600 + rng.integers(-262000, 262000, RX * CH) * 20
    c["code_incr"] = 6710886 * 40 + rng.integers(-10, 10, RX * CH)
    c["epoch_load"] = -1
    return c


def _run(gc, world, IF, cmds):
    from gnsscorr.trackshard import TrackShard, merge
    shards = [TrackShard(RX, CH, NS, rank=r, world=world, samp_rate=FS) for r in range(world)]
    out = []
    for k in range(CALLS):
        rows = IF[:, k * 2 * NS:(k + 1) * 2 * NS]
        for s in shards:
            s.load(rows)
            s.step(cmds[k])
        out.append(merge([s.results() for s in shards], RX * CH))
    return out


def test_sharded_union_equals_unsharded(gpu):
    rng = np.random.default_rng(31)
    sigs = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
                 doppler=float(rng.uniform(-3000, 3000)), cn0=48.0, data_bits=1)
            for p in rng.choice(np.arange(1, 33), 6, replace=False)]
    IF = np.stack([gpu.ifgen(CALLS * NS, sigs, fs=FS, seed=0x5EED0100 + r) for r in range(RX)])
    cmds = [_cmds(gpu, rng) for _ in range(CALLS)]
    one = _run(gpu, 1, IF, cmds)
    assert any((r["n_dumps"] > 0).any() for r in one)
    for world in (2, 3):
        many = _run(gpu, world, IF, cmds)
        for k in range(CALLS):
            assert one[k].tobytes() == many[k].tobytes(), (world, k)
