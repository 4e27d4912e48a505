"""bench.py's result line on CPU: every section's measurement stubbed with
placeholder numbers, main() must assemble and print the one JSON line with the
contract's keys (a KeyError or a renamed field there would only show on the GPU
box, at the driver's round-end run)."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _V(float):
    def __new__(cls, x=123456.789):   # printed like a real measurement (4 digits + exponent)
        return float.__new__(cls, x)


class _D(dict):
    def __missing__(self, k):
        return _V()


class _Dist:
    rank, world, local = 0, 1, 0

    def gather(self, x):
        return [x]

    def barrier(self):
        pass

    def max(self, x):
        return x

    def close(self):
        pass


def test_bench_main_assembles_the_json_line(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    monkeypatch.setattr(sys, "argv", ["bench.py", "--no-cpu-baseline"])
    monkeypatch.setattr(bench.gc, "lib", lambda: None)
    monkeypatch.setattr(bench.gc, "device_count", lambda: 1)
    monkeypatch.setattr(bench.gc, "pci_bus_id", lambda d: "0000:00:00.0")
    monkeypatch.setattr(bench.gc, "hip_runtime", lambda: "stub")
    monkeypatch.setattr(bench, "Dist", _Dist)
    lay = lambda: _D(channels=3072, ok=True)  # noqa: E731
    stubs = dict(
        run_acq=lambda *a, **k: _D(records=8, meta=_D(set_codes_ms=1.0), found=8, n_planted=8),
        run_track=lambda *a, **k: _D(steps=20, channels=3072, dumps_ok=True),
        run_track_io=lambda *a, **k: _D(steps=20, cs1_int8=lay(), cs1_packed2=lay(),
                                        rx12_packed2=lay(), host_int8=_D(channels=3072),
                                        host_packed2=_D(channels=3072),
                                        sim_gp2021_12ch=_D(nsamp=8184)),
        run_sgt=lambda *a, **k: _D(channels=3584, ok=True),
        run_fullsky=lambda *a, **k: _D(projection={"world_1_ms": 1.4}, found=12, n_planted=12),
        run_sdr=lambda *a, **k: _D(mw=_D(medium=_D(), weak=_D()), loop=_D(), long=_D(),
                                   bufs=None),
        run_glo_coherent=lambda *a, **k: _D(found=4, n_planted=4),
        run_gps_scilab=lambda *a, **k: _D(found=6, n_planted=6, nb=113, n=16000),
        run_acq_generic=lambda *a, **k: _D(found=8, n_planted=8, fs=38.192e6, n=38192))
    for k, v in stubs.items():
        monkeypatch.setattr(bench, k, v)
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.main()
    lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                "roofline"):
        assert key in d, key
    assert set(("bound", "achieved", "peak", "unit", "frac", "traffic")) <= set(d["roofline"])
    t = d["tracking"]
    assert t["roofline"]["calls_per_launch"] == bench.TRACK_CPL
    assert t["roofline"]["kernel_ms_per_launch"] == t["roofline"]["kernel_ms_per_call"] * \
        bench.TRACK_CPL
    assert t["closed_loop"]["kernel"] == bench.TRACK_KERNEL + " + osg_isr_kernel"
    assert t["closed_loop"]["launches_per_call"] == 2
    for lay_key in ("cs1_int8", "cs1_packed2", "rx12_packed2"):
        r = t["layouts"][lay_key]["roofline"]
        assert {"hbm_GBs", "hbm_frac", "traffic"} <= set(r), lay_key
    # the driver keeps the last ~8000 characters of stdout: the whole line must fit,
    # with room for the cpu_baseline objects (off here) and N=8 ranks; tracking last
    assert len(lines[0]) < 6800, len(lines[0])
    assert list(d)[-1] == "tracking"
    assert "glonass_tracking" in d and "fullsky" in d and "shard_projection" in d["fullsky"]


def test_bench_launches_n_ranks_itself():
    """`bench.py --gpus 2` without torch.distributed.run starts two rank processes
    that meet at the host-group barrier (BENCH_STUB: no library, no GPU)."""
    import subprocess
    env = dict(os.environ, BENCH_STUB="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "3", "--warmup", "1"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert sorted(r["rank"] for r in d["ranks"]) == [0, 1]
    assert [r["local_rank"] for r in d["ranks"]] == [0, 1]
    assert len({r["pid"] for r in d["ranks"]}) == 2
    assert d["max_rank"] == 1.0
    assert not any(r["torch_loaded"] for r in d["ranks"])   # no second HIP runtime
