"""CPU, multi-process: the N>1 control path over the host group
(gnsscorr/hostgroup.py: a Unix-domain socket on the node, no torch.distributed),
world sizes 2, 3 and 8.

* bench.Dist: barrier + max-over-ranks timing (the bench contract);
* full-sky sharding (gnsscorr/fullsky.py): every rank takes a disjoint group
  set, the per-group results are gathered (HostGroup.allgather) and
  merged on rank 0 in group order -- the only exchange config 5 needs;
* tracking sharding (gnsscorr/trackshard.py): channels round-robin over
  ranks, each rank's NCO commands remapped onto its local IF copies, results
  gathered by global channel index.
No GPU: each rank fabricates its shard's results.
"""
import os
import socket

import pytest
import multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "gnss-sdr.ru_amd")]
    import bench
    from gnsscorr.fullsky import GROUPS, merge, shard
    assert "torch" not in sys.modules
    d = bench.Dist()
    d.barrier()
    m = d.max(float(rank + 1) * 1.5)
    mine = shard(len(GROUPS), world, rank)
    part = [(i, GROUPS[i][0], GROUPS[i][1], float(i) * 10 + rank) for i in mine]
    allp = d.gather(part)
    if rank == 0:
        merged = merge(allp)
        q.put(("ok", m, [r[0] for r in merged], [r[3] for r in merged]))
    d.close()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_hostgroup_barrier_max_and_fullsky_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        tag, m, idx, vals = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert tag == "ok"
    assert m == 1.5 * world
    assert idx == list(range(46))
    assert vals == [i * 10.0 + i % world for i in range(46)]
    assert all(p.exitcode == 0 for p in procs)


def test_shard_is_a_partition():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "gnss-sdr.ru_amd"))
    from gnsscorr.fullsky import shard
    for world in (1, 2, 3, 4, 8):
        parts = [shard(46, world, r) for r in range(world)]
        flat = sorted(i for p in parts for i in p)
        assert flat == list(range(46))
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
    with pytest.raises(ValueError):
        shard(46, 2, 2)


def _track_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    import numpy as np
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "gnss-sdr.ru_amd")]
    import bench
    import gnsscorr as gc
    from gnsscorr.trackshard import local_cmds, merge, plan
    d = bench.Dist()
    n_rx, n_ch = 5, 12
    cmds = np.zeros(n_rx * n_ch, gc.NCO_CMD)
    cmds["prn"] = np.arange(n_rx * n_ch) % 32 + 1
    cmds["stream"] = np.repeat(np.arange(n_rx), n_ch)
    mine, streams, lstream = plan(n_rx, n_ch, world, rank)
    lc = local_cmds(cmds, mine, lstream)
    # every local channel reads the local copy of its own receiver's stream
    ok = all(streams[lc["stream"][i]] == cmds["stream"][g] for i, g in enumerate(mine))
    res = np.zeros(len(mine), gc.TRACK_RESULT)
    res["n_dumps"] = np.asarray(mine) * 3 + 1       # a per-channel fingerprint
    parts = d.gather((mine, res))
    if rank == 0:
        m = merge(parts, n_rx * n_ch)
        q.put(("ok", bool(ok), m["n_dumps"].tolist(), len(streams)))
    d.close()


@pytest.mark.parametrize("world", [2])
def test_hostgroup_track_sharding(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_track_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        tag, ok, dumps, nstreams = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert tag == "ok" and ok
    assert dumps == [g * 3 + 1 for g in range(60)]
    assert nstreams == 5                  # round-robin channels: every stream is copied
    assert all(p.exitcode == 0 for p in procs)


def test_track_plan_partition_and_merge_checks():
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "gnss-sdr.ru_amd"))
    import gnsscorr as gc
    from gnsscorr.trackshard import merge, plan
    for world in (1, 2, 3, 8):
        parts = [plan(7, 12, world, r)[0] for r in range(world)]
        assert sorted(g for p in parts for g in p) == list(range(84))
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
    with pytest.raises(RuntimeError):
        merge([([0, 1], np.zeros(2, gc.TRACK_RESULT))], 3)
    with pytest.raises(ValueError):
        plan(2, 12, 2, 5)


def test_track_shard_more_ranks_than_channels():
    """world > n_rx * n_ch: the surplus ranks hold no channels, build no context and
    contribute an empty part; the merge is still complete (no GPU touched)."""
    import sys
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "gnss-sdr.ru_amd"))
    import gnsscorr as gc
    from gnsscorr.trackshard import TrackShard, merge, plan
    world = 5
    parts = [plan(1, 3, world, r) for r in range(world)]
    assert [len(p[0]) for p in parts] == [1, 1, 1, 0, 0]
    idle = TrackShard(1, 3, 16368, rank=4, world=world)
    assert idle.ctx is None
    idle.load(np.zeros((1, 2 * 16368), np.int8))
    idle.step(np.zeros(3, gc.NCO_CMD))
    ids, res = idle.results()
    assert ids == [] and len(res) == 0
    full = [(p[0], np.zeros(len(p[0]), gc.TRACK_RESULT)) for p in parts]
    assert len(merge(full, 3)) == 3


def _group_worker(rank, world, key, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "gnss-sdr.ru_amd")]
    from gnsscorr.hostgroup import HostGroup
    g = HostGroup(rank, world, key=key, timeout_s=60)
    out = []
    for k in range(20):          # back-to-back collectives keep their order
        out.append(g.allgather((rank, k)))
        assert g.max(rank * k) == (world - 1) * k
    g.close()
    q.put((rank, out))


def test_hostgroup_repeated_collectives_and_stale_socket(tmp_path):
    """20 gathers in a row arrive in order on every rank; a socket file left by a
    crashed run under the same key is replaced, not connected to."""
    import tempfile
    key = f"test-{os.getpid()}"
    stale = os.path.join(tempfile.gettempdir(), f"gnsscorr-{key}.sock")
    open(stale, "w").close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    world = 4
    procs = [ctx.Process(target=_group_worker, args=(r, world, key, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(world):
        assert got[r] == [[(i, k) for i in range(world)] for k in range(20)]
    assert not os.path.exists(stale)
