"""Host-side process group for the N-rank paths: barrier, max and
all-gather of small Python objects between the ranks of ONE node.

The sharded paths (gnsscorr/fullsky.py, gnsscorr/trackshard.py, bench.py --gpus N)
exchange nothing on the data path: each rank searches or tracks its own shard on
its own GPU, and the only exchange is the final gather of a few hundred result
rows plus the bench's barrier and max-over-ranks timing.  That needs no RCCL and
no torch.distributed: rank 0 listens on a Unix-domain socket, the other ranks
connect, and every collective is a star (send to rank 0, rank 0 sends the list
back).  So no rank imports torch, and the only HIP runtime a rank maps is the one
libgnsscorr.so was built against (the gloo transport pulled in
torch's own libamdhip64 beside it).

Rendezvous: the socket path is derived from a key every rank of one job shares:
GNSSCORR_GROUP_KEY if set (bench.py's own launcher sets it), else MASTER_PORT and
TORCHELASTIC_RUN_ID (torch.distributed.run holds MASTER_PORT for the job's life,
so two concurrent jobs never share a key).
"""
import os
import tempfile
import time
from multiprocessing.connection import Client, Listener


def group_key() -> str:
    k = os.environ.get("GNSSCORR_GROUP_KEY")
    if k:
        return k
    return "%s-%s" % (os.environ.get("MASTER_PORT", "0"),
                      os.environ.get("TORCHELASTIC_RUN_ID", "none"))


class HostGroup:
    """world ranks on one node; rank 0 hosts the socket.  timeout_s bounds the
    rendezvous (a rank that never arrives ends the job with an error)."""

    def __init__(self, rank: int, world: int, key: str = None, timeout_s: float = 600.0):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world = rank, world
        self.conns, self.conn, self.listener = [], None, None
        if world == 1:
            return
        key = key or group_key()
        self.path = os.path.join(tempfile.gettempdir(), f"gnsscorr-{key}.sock")
        auth = ("gnsscorr-" + key).encode()
        if rank == 0:
            try:
                os.unlink(self.path)        # a socket file a crashed run left behind
            except FileNotFoundError:
                pass
            self.listener = Listener(self.path, family="AF_UNIX", authkey=auth)
            self.conns = [None] * world
            for _ in range(world - 1):
                c = self.listener.accept()
                r = c.recv()
                if not (0 < r < world) or self.conns[r] is not None:
                    raise RuntimeError(f"hostgroup: bad or duplicate rank {r}")
                self.conns[r] = c
        else:
            t_end = time.monotonic() + timeout_s
            while True:
                try:
                    self.conn = Client(self.path, family="AF_UNIX", authkey=auth)
                    break
                except (FileNotFoundError, ConnectionRefusedError):
                    if time.monotonic() > t_end:
                        raise TimeoutError(f"hostgroup: rank 0 never listened on {self.path}")
                    time.sleep(0.02)
            self.conn.send(rank)

    def allgather(self, obj):
        """Every rank's object, in rank order, on every rank."""
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [c.recv() for c in self.conns[1:]]
            for c in self.conns[1:]:
                c.send(out)
            return out
        self.conn.send(obj)
        return self.conn.recv()

    def barrier(self):
        self.allgather(None)

    def max(self, x: float) -> float:
        return max(self.allgather(float(x)))

    def close(self):
        if self.world == 1:
            return
        # a last barrier: rank 0 must not remove the socket while others still talk
        try:
            self.barrier()
        finally:
            for c in self.conns[1:] + [self.conn]:
                if c is not None:
                    c.close()
            if self.listener is not None:
                self.listener.close()   # also removes the socket file
            self.conns, self.conn, self.listener = [], None, None
