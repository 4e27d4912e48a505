"""bench.py -- BASELINE.json metric on MI355X:
"1ms E/P/L correlations/sec + acquisition cells/sec @16.368Msps; 1/2/4/8 GPU".

Primary line (`value`): acquisition cells/s on BASELINE config 2 -- a full
32-PRN x 41-Doppler-bin cold-start search (acquisition.sci semantics: 1 ms
coherent, two consecutive 1-ms blocks, keep the better), 16368 samples per
code period, computed in fp64 like the reference (Scilab doubles; parity
~1e-12 relative, tests/test_acq_gpu.py).  A step = complete searches of
ACQ_RECORDS (16) consecutive 2-ms IF records already resident in HBM, each exactly
one acquisition.sci search (classes, wipe-off + FFT of the class rows, 2624
correlation IFFTs, peak/second-peak/metric for 32 PRNs), run as one launch per
stage (gnsscorr_acq_set_records): one record fills the GPU for 10.25 rounds of
units, so a single search leaves most CUs idle in its last round.
Weak scaling: every rank runs its own search on its own record each step (PRN
x Doppler cells shard with no exchange step: no collective on the data path).
The fp32 fast path is reported beside it as `acquisition_f32`.

Secondary object (`tracking`): 1-ms E/P/L correlations per second --
256 receivers x 12 GP2021 channels (BASELINE config 3 scaled out), each
receiver on its own 16.368 Msps int8 IQ stream in HBM, one 1-ms correlator
call per step (NCO words replayed from a command schedule: the DLL/PLL is
host code and not part of the hot path).

Run: python bench.py [--gpus N --steps K --warmup W].  For N>1 under
torch.distributed.run the launcher's RANK/WORLD_SIZE env is used; without it
bench.py starts the N rank processes itself (launch_ranks).  Ranks synchronise
over a host socket (gnsscorr/hostgroup.py, no torch.distributed) only for the
barrier, the max-over-ranks time and a small result gather.

Output: ONE JSON line on rank 0 -- the contract's keys first, then every
secondary section without its descriptive strings (floats to 4 significant
digits), tracking lines last; the full result, descriptions included, goes to
gpurun_out/bench_detail.json.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnss-sdr.ru_amd"))
import gnsscorr as gc  # noqa: E402

FS = 16.368e6
N = 16368
N_PRN, N_BINS, N_BLK = 32, 41, 2
ACQ_RECORDS = int(os.environ.get("BENCH_ACQ_RECORDS", "16"))   # config-2 searches per launch (gnsscorr_acq_set_records, fp64)
CELLS_PER_SEARCH = N_PRN * N_BINS * N          # 21,474,816
# algorithmic FLOPs of one correlation cell per 1-ms block: radix-2-equivalent
# IFFT 5*log2(N) + complex multiply 6 + |.|^2 3 + max 1  
FLOP_PER_CELL_BLOCK = 5.0 * np.log2(N) + 6 + 3 + 1
PEAK_FP32_TFLOPS = 157.3                       # MI355X_MICROARCH.md (vector == matrix f32)
ACQ64_KERNEL = "acq64_corr_kernel<Plan<16368, 16, 33, 31, 512, true>, 0, false>"  # best-of-blocks
PEAK_HBM_GBS = 8000.0
# the OSG tracking correlator of IQ streams (track.hip osg_stream_kernel<packed, waves/channel>)
TRACK_KERNEL = "osg_stream_kernel<false, false>"      # int8 IQ, open loop
TRACK_KERNEL_PK = "osg_stream_kernel<true, false>"    # 2-bit packed IQ
TRACK_KERNEL_CL = "osg_stream_kernel<false, true>"    # closed loop, GNSSCORR_OSG_FUSED=1: gpsisr fused
# calls per osg_stream_kernel launch in the tracking lines (replay and closed loop run
# n calls per launch; a fixed count keeps rocprof per-launch figures comparable)
TRACK_CPL = 10
PEAK_INT_TOPS = 78.6                           # 256 CU x 128 lanes x 2.4 GHz, 32-bit VALU
# 1024 receivers x 12 channels per GPU: 12288 channel-waves give 4 waves per SIMD
# (3072 give 3; the kernel is latency bound there: rx12 int8 29-30 -> 24-25 us per
# 3072 channel-ms at 12288, same box, profiles/r5/fullsky_join_and_trk_scan_r5c.log)
TRACK_RX, TRACK_CH, TRACK_NS = 1024, 12, 16368
TRACK_C1 = TRACK_RX * TRACK_CH   # channels of the one-stream-per-channel layouts
TRACK_RX_HOST = 256              # receivers of the PCIe-inclusive host-buffer lines
SGT_RX, SGT_FS = 256, 16.0e6                   # GLONASS records: initSettings.sci fs = 16 MHz
SGT_DP_PER_SAMPLE = 27                         # fp64 ops/sample of sgt_track_kernel
PEAK_FP64_TFLOPS = 78.6                        # MI355X FP64 vector (AMD spec; not in the guide)
TRACK_OPS_PER_SAMPLE = 20                      # SURVEY 8d integer-op model
EV_EVERY = 1                                   # kernel-timed steps: 1 of EV_EVERY (every step)
METRIC = "1ms E/P/L correlations/sec + acquisition cells/sec @16.368Msps; 1/2/4/8 GPU"


class Dist:
    """The bench's ranks: barrier, max-over-ranks and gather over gnsscorr.hostgroup (a
    Unix-domain socket on the node, no torch.distributed), so a rank maps no HIP
    runtime but the one libgnsscorr.so was built against."""

    def __init__(self, load_lib=True):
        from gnsscorr.hostgroup import HostGroup
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.group = HostGroup(self.rank, self.world)

    def barrier(self):
        self.group.barrier()

    def max(self, x: float) -> float:
        return self.group.max(x)

    def gather(self, obj):
        """All ranks' objects (list, rank order); small host data only."""
        return self.group.allgather(obj)

    def close(self):
        self.group.close()


def acq_setup(dev, rank, precision=gc.ACQ_F64, records=1):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    rng = np.random.default_rng(100 + rank)
    planted = rng.choice(np.arange(1, 33), 8, replace=False)
    sigs = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
                 doppler=float(rng.uniform(-5000, 5000)), cn0=49.0, data_bits=1) for p in planted]
    # `records` consecutive 2-ms records of the same receiver stream
    IF = gc.ifgen(records * N_BLK * N, sigs, fs=FS, seed=0x5EED0002 + rank)
    codes = np.stack([gc.sample_code(gc.ca_code(p), 1.023e6, FS, N) for p in range(1, 33)])
    freqs = 2.42e6 - 10000.0 + 500.0 * np.arange(N_BINS)           # acquisition.sci:101-104
    ctx = gc.AcqCtx(FS, N, device=dev, max_freqs=N_BINS, max_blocks=N_BLK * records,
                    max_codes=N_PRN, precision=precision)
    # acquisition.sci:91-95 makes caCodesTable and takes conj(fft(caCodesTable(PRN,:)))
    # inside every search; here the 32 replicas are generated on the device from the
    # PRN list and transformed (gnsscorr_acq_set_prn_codes) once, outside the timed
    # steps: 32 of the ~2 700 transforms of a search.  The context's first call is
    # timed here (gnsscorr_acq_create did the one-time work: chip table, buffers,
    # code objects loaded); the warm
    # cost and a whole cold-start search with the codes inside it are timed in
    # run_acq (single_search.with_codes).
    t0 = time.perf_counter()
    ctx.set_prn_codes(np.arange(1, N_PRN + 1, dtype=np.int32))
    ctx.sync()
    set_codes_ms = (time.perf_counter() - t0) * 1e3
    if records > 1:
        ctx.set_records(records)
    bufs = dict(
        d_if=gc.DevBuf.from_array(IF, dev), d_freqs=gc.DevBuf.from_array(freqs, dev),
        d_gcode=gc.DevBuf.from_array(np.arange(N_PRN, dtype=np.int32), dev),
        d_gfreq=gc.DevBuf.from_array(np.tile(np.arange(N_BINS, dtype=np.int32), N_PRN), dev),
        d_rows=gc.DevBuf(records * N_PRN * N_BINS * gc.ACQ_ROW.itemsize, dev),
        d_res=gc.DevBuf(records * N_PRN * gc.ACQ_RESULT.itemsize, dev))
    return ctx, bufs, dict(IF=IF[:2 * N_BLK * N], codes=codes, freqs=freqs, planted=planted,
                           records=records, set_codes_ms=set_codes_ms)


def acq_step(ctx, b, ev=None):
    ctx.spectra_dev(b["d_if"].ptr, N_BLK, N_BINS, b["d_freqs"].ptr)
    if ev:
        ev[0].record(ctx.stream)
    # the correlation kernel alone between the events (row statistics stay in
    # the context), then the per-PRN selection kernel (acquisition.sci:126-186)
    ctx.correlate_dev(N_BLK, b["d_freqs"].ptr, N_PRN, N_BINS, b["d_gcode"].ptr, b["d_gfreq"].ptr)
    if ev:
        ev[1].record(ctx.stream)
    ctx.select_dev(N_PRN, N_BINS, b["d_freqs"].ptr, b["d_gfreq"].ptr, b["d_rows"].ptr,
                   b["d_res"].ptr)


def run_acq(dist, dev, steps, warmup, precision=gc.ACQ_F64, records=None):
    if records is None:
        records = ACQ_RECORDS if precision == gc.ACQ_F64 else 1
    ctx, b, meta = acq_setup(dev, dist.rank, precision, records)
    for _ in range(warmup):
        acq_step(ctx, b)
    ctx.sync()
    # correctness guard: the planted PRNs must be found in every record (cheap,
    # outside timing)
    res = b["d_res"].download(gc.ACQ_RESULT).reshape(records, N_PRN)
    found = sum(1 for r in range(records) for p in meta["planted"] if res[r][p - 1]["metric"] > 2.5)
    # kernel timing on every EV_EVERY-th step.  Every step: the clocks are still
    # ramping over the first ~40 launches (1.58 -> 1.43 ms per 8-record launch,
    # tools/acq_step_times.py), so a sample of steps 0 and 10 read ~2.5 % above the
    # timed region's mean; the event pair costs no measurable step time
    ev_steps = list(range(0, steps, EV_EVERY))
    evs = {k: (gc.Event(dev), gc.Event(dev)) for k in ev_steps}
    dist.barrier()
    gc.dev_synchronize(dev)
    t0 = time.perf_counter()
    for k in range(steps):
        acq_step(ctx, b, evs.get(k))
    ctx.sync()
    gc.dev_synchronize(dev)
    t1 = time.perf_counter()
    dist.barrier()
    dt = dist.max(t1 - t0)
    corr_ms = float(np.mean([a.elapsed_ms(z) for a, z in evs.values()]))
    with_codes = None
    if records == 1:
        # the cold start with the code spectra inside it (acquisition.sci:91-95 per
        # search), warm context: codes generated on the device + spectra alone, then
        # the whole search, each ended by a host sync (the wall a caller waits)
        ids = np.arange(1, N_PRN + 1, dtype=np.int32)
        for _ in range(3):
            ctx.set_prn_codes(ids)
            acq_step(ctx, b)
        ctx.sync()
        lat_c, lat_s = [], []
        for _ in range(steps):
            t0 = time.perf_counter()
            ctx.set_prn_codes(ids)
            ctx.sync()
            lat_c.append(time.perf_counter() - t0)
        for _ in range(steps):
            t0 = time.perf_counter()
            ctx.set_prn_codes(ids)
            acq_step(ctx, b)
            ctx.sync()
            lat_s.append(time.perf_counter() - t0)
        res = b["d_res"].download(gc.ACQ_RESULT).reshape(records, N_PRN)
        with_codes = dict(
            code_spectra_ms=dist.max(float(np.mean(lat_c)) * 1e3),
            ms_wall=dist.max(float(np.mean(lat_s)) * 1e3),
            p99_ms=dist.max(float(np.percentile(lat_s, 99)) * 1e3),
            found=sum(1 for p in meta["planted"] if res[0][p - 1]["metric"] > 2.5))
    return dict(dt=dt, corr_ms=dist.max(corr_ms), found=found,
                n_planted=len(meta["planted"]) * records, records=records, meta=meta,
                with_codes=with_codes)


GENERIC_FS = 38.192e6   # the classic SoftGNSS front end (acquisition.sci: samplesPerCode 38192)


GENERIC_RECORDS = int(os.environ.get("BENCH_GENERIC_RECORDS", "16"))   # searches per step (as ACQ_RECORDS)


def run_acq_generic(dist, dev, steps, warmup, fs=GENERIC_FS, records=None):
    """Config 2's search at a rate without a compiled plan: the generic fp64 engine
    (38192 = 112 x 341: the four-step plan, the correlation product fused into the
    column pass and |.|^2 with the row statistics into the row pass), `records`
    consecutive 2-ms records of one stream per step (gnsscorr_acq_set_records, as the
    config-2 line): ms per search = step time / records."""
    records = GENERIC_RECORDS if records is None else records
    n = int(round(fs / 1000.0))
    spc = int(round(fs / 1.023e6))   # samplesPerCodeChip (GPS/L1/acquisition.sci:147), the exclusion window
    rng = np.random.default_rng(300 + dist.rank)
    planted = rng.choice(np.arange(1, 33), 8, replace=False)
    sigs = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
                 doppler=float(rng.uniform(-5000, 5000)), cn0=49.0, data_bits=1) for p in planted]
    IF = gc.ifgen(records * N_BLK * n, sigs, fs=fs, seed=0x5EED0030 + dist.rank)
    codes = np.stack([gc.sample_code(gc.ca_code(p), 1.023e6, fs, n) for p in range(1, 33)])
    freqs = 2.42e6 - 10000.0 + 500.0 * np.arange(N_BINS)
    ctx = gc.AcqCtx(fs, n, device=dev, max_freqs=N_BINS, max_blocks=N_BLK * records,
                    max_codes=N_PRN)
    ctx.set_codes(codes)
    if records > 1:
        ctx.set_records(records)
    b = dict(d_if=gc.DevBuf.from_array(IF, dev), d_freqs=gc.DevBuf.from_array(freqs, dev),
             d_gcode=gc.DevBuf.from_array(np.arange(N_PRN, dtype=np.int32), dev),
             d_gfreq=gc.DevBuf.from_array(np.tile(np.arange(N_BINS, dtype=np.int32), N_PRN), dev),
             d_rows=gc.DevBuf(records * N_PRN * N_BINS * gc.ACQ_ROW.itemsize, dev),
             d_res=gc.DevBuf(records * N_PRN * gc.ACQ_RESULT.itemsize, dev))

    def step():
        ctx.spectra_dev(b["d_if"].ptr, N_BLK, N_BINS, b["d_freqs"].ptr)
        ctx.correlate_dev(N_BLK, b["d_freqs"].ptr, N_PRN, N_BINS, b["d_gcode"].ptr,
                          b["d_gfreq"].ptr, spc=spc)
        ctx.select_dev(N_PRN, N_BINS, b["d_freqs"].ptr, b["d_gfreq"].ptr, b["d_rows"].ptr,
                       b["d_res"].ptr)

    for _ in range(warmup):
        step()
    ctx.sync()
    res = b["d_res"].download(gc.ACQ_RESULT).reshape(records, N_PRN)
    found = sum(1 for r in range(records) for p in planted if res[r][p - 1]["metric"] > 2.5)
    dist.barrier()
    gc.dev_synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    gc.dev_synchronize(dev)
    dt = dist.max(time.perf_counter() - t0)
    return dict(dt=dt, steps=steps, n=n, fs=fs, found=found, n_planted=records * len(planted),
                records=records)


def _track_steps(steps):
    """timed calls rounded up to whole TRACK_CPL-call launches"""
    return -(-steps // TRACK_CPL) * TRACK_CPL


def _replay_launches(ctx, d_if, stride, if_step_bytes, d_cmds, d_res, C, start, n):
    """calls [start, start + n) as launches of TRACK_CPL consecutive calls each"""
    for s in range(start, start + n, TRACK_CPL):
        m = min(TRACK_CPL, start + n - s)
        ctx.replay_dev(d_if.ptr + s * if_step_bytes, stride, TRACK_NS, m,
                       d_cmds.ptr + s * C * gc.NCO_CMD.itemsize,
                       d_res.ptr + s * C * gc.TRACK_RESULT.itemsize)


def run_track(dist, dev, steps, warmup):
    """The main tracking line: 256 receivers x 12 channels, 1-ms calls replayed on the
    device, TRACK_CPL calls per launch; warmup: one launch (warmup is rounded to it)."""
    C = TRACK_RX * TRACK_CH
    steps = _track_steps(steps)
    warmup = TRACK_CPL
    K = steps + warmup
    stride = K * TRACK_NS                                        # samples per stream
    d_if = gc.DevBuf(TRACK_RX * stride * 2, dev)
    d_if.fill_if2(0x5EED0003 + dist.rank)
    rng = np.random.default_rng(7 + dist.rank)
    cmd1 = np.zeros(C, gc.NCO_CMD)
    cmd1["prn"] = rng.integers(1, 33, C)
    cmd1["stream"] = np.repeat(np.arange(TRACK_RX), TRACK_CH)
    cmd1["carrier_incr"] = 635008600 + rng.integers(-262000, 262000, C) * 20   # +-5 kHz
    cmd1["code_incr"] = 6710886 * 40 + rng.integers(-800, 800, C)   # +-3 ppm code Doppler
    cmd1["epoch_load"] = -1
    cmds = np.tile(cmd1, K)
    d_cmds = gc.DevBuf.from_array(cmds, dev)
    d_res = gc.DevBuf(K * C * gc.TRACK_RESULT.itemsize, dev)
    ctx = gc.TrackCtx(C, iq=True, device=dev, max_nsamp=TRACK_NS, samp_rate=FS)
    step_b = ctx.if_bytes(TRACK_NS)
    _replay_launches(ctx, d_if, stride, step_b, d_cmds, d_res, C, 0, warmup)
    ctx.sync()
    e0, e1 = gc.Event(dev), gc.Event(dev)
    dist.barrier()
    gc.dev_synchronize(dev)
    t0 = time.perf_counter()
    e0.record(ctx.stream)
    _replay_launches(ctx, d_if, stride, step_b, d_cmds, d_res, C, warmup, steps)
    e1.record(ctx.stream)
    ctx.sync()
    gc.dev_synchronize(dev)
    t1 = time.perf_counter()
    dist.barrier()
    dt = dist.max(t1 - t0)
    kern_ms = dist.max(e0.elapsed_ms(e1) / steps)
    res = d_res.download(gc.TRACK_RESULT, C, (K - 1) * C * gc.TRACK_RESULT.itemsize)
    dumps_ok = bool((res["n_dumps"] >= 0).all() and (res["n_dumps"] <= 2).all())
    # closed loop on the device: correlator + gpsisr channel loops per call, no host
    cfg = gc.osg_loop_cfg(samp_rate=FS)
    loops, cl_cmds = gc.osg_loop_reset(cfg, cmd1["prn"])
    cl_cmds["stream"] = cmd1["stream"]
    d_l, d_c = gc.DevBuf.from_array(loops, dev), gc.DevBuf.from_array(cl_cmds, dev)
    d_rh = gc.DevBuf(K * C * gc.TRACK_RESULT.itemsize, dev)
    ctx2 = gc.TrackCtx(C, iq=True, device=dev, max_nsamp=TRACK_NS, samp_rate=FS)

    def closed(start, n):
        for s0 in range(start, start + n, TRACK_CPL):
            m = min(TRACK_CPL, start + n - s0)
            gc.osg_closed_loop_dev(ctx2, cfg, d_if.ptr + s0 * step_b, stride, TRACK_NS, m, C,
                                   d_l.ptr, d_c.ptr, d_rh.ptr + s0 * C * gc.TRACK_RESULT.itemsize)
    closed(0, warmup)
    ctx2.sync()
    dist.barrier()
    t0 = time.perf_counter()
    e0.record(ctx2.stream)
    closed(warmup, steps)
    e1.record(ctx2.stream)
    ctx2.sync()
    dt_cl = dist.max(time.perf_counter() - t0)
    cl_ms = dist.max(e0.elapsed_ms(e1) / steps)
    return dict(dt=dt, kern_ms=kern_ms, channels=C, dumps_ok=dumps_ok, dt_cl=dt_cl, cl_ms=cl_ms,
                steps=steps)


def _replay_timed(dist, dev, ctx, d_if, stride, if_step_bytes, d_cmds, d_res, C, steps, warmup):
    """warmup + steps replayed 1-ms calls (TRACK_CPL per launch; the caller sizes the
    buffers for warmup + steps calls); returns (wall s, kernel ms per call, results)."""
    _replay_launches(ctx, d_if, stride, if_step_bytes, d_cmds, d_res, C, 0, warmup)
    ctx.sync()
    e0, e1 = gc.Event(dev), gc.Event(dev)
    dist.barrier()
    gc.dev_synchronize(dev)
    t0 = time.perf_counter()
    e0.record(ctx.stream)
    _replay_launches(ctx, d_if, stride, if_step_bytes, d_cmds, d_res, C, warmup, steps)
    e1.record(ctx.stream)
    ctx.sync()
    gc.dev_synchronize(dev)
    dt = dist.max(time.perf_counter() - t0)
    res = d_res.download(gc.TRACK_RESULT, C, (warmup + steps - 1) * C * gc.TRACK_RESULT.itemsize)
    return dt, dist.max(e0.elapsed_ms(e1) / steps), res


def _track_cmds(rng, C, streams):
    cmd1 = np.zeros(C, gc.NCO_CMD)
    cmd1["prn"] = rng.integers(1, 33, C)
    cmd1["stream"] = streams
    cmd1["carrier_incr"] = 635008600 + rng.integers(-262000, 262000, C) * 20   # +-5 kHz
    cmd1["code_incr"] = 6710886 * 40 + rng.integers(-800, 800, C)   # +-3 ppm code Doppler
    cmd1["epoch_load"] = -1
    return cmd1


def run_track_io(dist, dev, steps, warmup):
    """Tracking layouts beside the main line (all 16.368 Msps, 1-ms calls):
    * one IF stream PER CHANNEL (C_s = 1: the layout where HBM bytes bind), int8 and
      2-bit packed (GNSSCORR_IF_PACKED2), TRACK_C1 channels, distinct data every call;
    * the main 256 x 12 layout with packed streams;
    * PCIe-inclusive: gnsscorr_track from host buffers (256 x 12 channels per call);
    * config 3 as the reference runs it: 12 channels, Sim_GP2021_int per 512-us
      interrupt (osgnss_next_step.c:150,168-184) through the legacy shim, per-call latency."""
    out = {}
    steps = _track_steps(steps)
    warmup = TRACK_CPL
    K = steps + warmup
    rng = np.random.default_rng(17 + dist.rank)
    C1 = TRACK_C1
    for packed in (False, True):
        stride = K * TRACK_NS
        bytes_stream = stride * 2 // (4 if packed else 1)
        d_if = gc.DevBuf(C1 * bytes_stream, dev)
        d_if.fill_if2(0x5EED000B + dist.rank)      # any byte is a valid packed code
        cmd1 = _track_cmds(rng, C1, np.arange(C1))
        d_cmds = gc.DevBuf.from_array(np.tile(cmd1, K), dev)
        d_res = gc.DevBuf(K * C1 * gc.TRACK_RESULT.itemsize, dev)
        ctx = gc.TrackCtx(C1, iq=True, device=dev, max_nsamp=TRACK_NS, samp_rate=FS,
                          packed=packed)
        ctx.set_layout(True)   # every channel has its own stream (no effect on packed ones)
        dt, kms, res = _replay_timed(dist, dev, ctx, d_if, stride, ctx.if_bytes(TRACK_NS),
                                     d_cmds, d_res, C1, steps, warmup)
        out["cs1_packed2" if packed else "cs1_int8"] = dict(
            dt=dt, kern_ms=kms, channels=C1, bytes_launch=C1 * (ctx.if_bytes(TRACK_NS) + 64),
            ok=bool((res["n_dumps"] >= 0).all() and (res["n_dumps"] <= 2).all()))
        ctx.close()
        d_if.free()
    # main layout, packed
    C = TRACK_RX * TRACK_CH
    stride = K * TRACK_NS
    d_if = gc.DevBuf(TRACK_RX * stride // 2, dev)
    d_if.fill_if2(0x5EED000C + dist.rank)
    cmd1 = _track_cmds(rng, C, np.repeat(np.arange(TRACK_RX), TRACK_CH))
    d_cmds = gc.DevBuf.from_array(np.tile(cmd1, K), dev)
    d_res = gc.DevBuf(K * C * gc.TRACK_RESULT.itemsize, dev)
    ctx = gc.TrackCtx(C, iq=True, device=dev, max_nsamp=TRACK_NS, samp_rate=FS, packed=True)
    dt, kms, res = _replay_timed(dist, dev, ctx, d_if, stride, ctx.if_bytes(TRACK_NS), d_cmds,
                                 d_res, C, steps, warmup)
    out["rx12_packed2"] = dict(dt=dt, kern_ms=kms, channels=C,
                               bytes_launch=C * (ctx.if_bytes(TRACK_NS) / TRACK_CH + 64))
    ctx.close()
    d_if.free()
    # PCIe-inclusive: host IF (pageable numpy) -> gnsscorr_track -> host results, per call
    Ch = TRACK_RX_HOST * TRACK_CH
    cmdh = _track_cmds(rng, Ch, np.repeat(np.arange(TRACK_RX_HOST), TRACK_CH))
    for packed in (False, True):
        ctx = gc.TrackCtx(Ch, iq=True, device=dev, max_nsamp=TRACK_NS, samp_rate=FS, packed=packed)
        h_if = np.random.default_rng(3).integers(-128, 128, TRACK_RX_HOST * ctx.if_bytes(TRACK_NS),
                                                 dtype=np.int8)
        if not packed:
            h_if = np.random.default_rng(3).choice(np.array([-3, -1, 1, 3], np.int8), h_if.size)
        n_calls = max(steps, 20)
        for _ in range(3):
            ctx.track(h_if, TRACK_NS, cmdh, n_streams=TRACK_RX_HOST, stream_stride=TRACK_NS)
        lat = []
        dist.barrier()
        for _ in range(n_calls):
            t0 = time.perf_counter()
            ctx.track(h_if, TRACK_NS, cmdh, n_streams=TRACK_RX_HOST, stream_stride=TRACK_NS)
            lat.append(time.perf_counter() - t0)
        lat = np.array(lat)
        out["host_packed2" if packed else "host_int8"] = dict(
            channels=Ch, calls=n_calls, mean_ms=dist.max(float(lat.mean()) * 1e3),
            p99_ms=dist.max(float(np.percentile(lat, 99)) * 1e3),
            h2d_bytes=TRACK_RX_HOST * ctx.if_bytes(TRACK_NS))
        ctx.close()
    # config 3 through the legacy shim: 12 channels, 512-us interrupts
    ns = int(FS * 512 / 1.0e6)                   # osgnss_next_step.c:150 (nsamp = fs*interr_int)
    osg = gc.OSG(samp_rate=FS, n_channels=12, use_iq=True, device=dev)
    osg.correlator_init(0.0)
    for ch in range(12):
        osg.ch_cntl(ch, ch + 1)
        osg.ch_carrier(ch, osg.gps_carrier_ref + 300 * ch)
        osg.ch_code(ch, osg.gps_code_ref)
    IF12 = np.random.default_rng(4).choice(np.array([-3, -1, 1, 3], np.int8), 2 * ns * 64)
    n_calls = 2000
    for k in range(20):
        osg.sim(IF12[(k % 64) * 2 * ns:], ns)
    lat = np.empty(n_calls)
    for k in range(n_calls):
        chunk = IF12[(k % 64) * 2 * ns:(k % 64 + 1) * 2 * ns]
        t0 = time.perf_counter()
        osg.sim(chunk, ns)
        lat[k] = time.perf_counter() - t0
    out["sim_gp2021_12ch"] = dict(nsamp=ns, calls=n_calls, budget_us=512.0,
                                  mean_us=float(lat.mean() * 1e6),
                                  p50_us=float(np.percentile(lat, 50) * 1e6),
                                  p99_us=float(np.percentile(lat, 99) * 1e6),
                                  max_us=float(lat.max() * 1e6))
    out["steps"] = steps
    return out


def run_sgt(dist, dev, steps, warmup, fs=SGT_FS):
    """BASELINE config 4: GLONASS L1OF 14 FDMA channels, tracking.sci float loop on the GPU.
    Throughput: SGT_RX records x 14 FCH; latency: one 14-channel receiver.  fs: the
    Scilab receiver's 16 MHz (initSettings.sci) or config 4's 16.368 Msps."""
    K = steps + warmup + 2
    ns = int(fs * K / 1000)
    stride = 2 * ns
    d_if = gc.DevBuf(SGT_RX * stride, dev)
    d_if.fill_if2(0x5EED0004 + dist.rank)
    ctx = gc.SgtCtx(1, device=dev, samplingFreq=fs)
    rng = np.random.default_rng(44 + dist.rank)
    fch = np.tile(np.arange(-7, 7), SGT_RX)
    C = len(fch)
    ch = ctx.init_chans(fch, rng.integers(1, 16000, C), 1e6 + 0.5625e6 * fch +
                        rng.uniform(-3000, 3000, C), streams=np.repeat(np.arange(SGT_RX), 14))
    d_ch = gc.DevBuf.from_array(ch, dev)
    d_ep = gc.DevBuf(C * max(steps, warmup) * gc.SGT_EPOCH.itemsize, dev)
    ctx.track_dev(d_if.ptr, stride, ns, C, d_ch.ptr, warmup, d_ep.ptr)
    ctx.sync()
    e0, e1 = gc.Event(dev), gc.Event(dev)
    dist.barrier()
    gc.dev_synchronize(dev)
    t0 = time.perf_counter()
    e0.record(ctx.stream)
    ctx.track_dev(d_if.ptr, stride, ns, C, d_ch.ptr, steps, d_ep.ptr)
    e1.record(ctx.stream)
    ctx.sync()
    t1 = time.perf_counter()
    dist.barrier()
    dt = dist.max(t1 - t0)
    kern_ms = dist.max(e0.elapsed_ms(e1))
    ep = d_ep.download(gc.SGT_EPOCH, C * steps).reshape(C, steps)
    ok = bool((ep["status"] == 0).all() and
              (np.abs(ep["blksize"] - round(fs / 1000)) < 20).all())
    # config 4 as stated: one 14-channel receiver, epochs back to back
    ch14 = ctx.init_chans(np.arange(-7, 7), rng.integers(1, 16000, 14),
                          1e6 + 0.5625e6 * np.arange(-7, 7))
    d14 = gc.DevBuf.from_array(ch14, dev)
    ctx.track_dev(d_if.ptr, stride, ns, 14, d14.ptr, warmup, d_ep.ptr)
    ctx.sync()          # DevBuf copies are not ordered against the context stream
    d14.upload(ch14)
    e0.record(ctx.stream)
    ctx.track_dev(d_if.ptr, stride, ns, 14, d14.ptr, steps, d_ep.ptr)
    e1.record(ctx.stream)
    ctx.sync()
    lat_ms = e0.elapsed_ms(e1) / steps
    return dict(dt=dt, kern_ms=kern_ms, channels=C, steps=steps, ok=ok, lat_ms=lat_ms, fs=fs)


def run_fullsky(dist, dev, steps, warmup):
    """BASELINE config 5: 32 GPS + 14 GLONASS FCH x 41 bins, 10 ms non-coherent, one full-sky
    search per step split over the ranks (strong scaling; groups sharded, no data exchange)."""
    from gnsscorr.fullsky import FullSky, merge
    rng = np.random.default_rng(0x5EED0005)
    gps = rng.choice(np.arange(1, 33), 8, replace=False)
    glo = rng.choice(np.arange(-7, 7), 4, replace=False)
    sg = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
               doppler=float(rng.uniform(-5000, 5000)), cn0=42.0, data_bits=1) for p in gps]
    sl = [dict(system=1, fch=int(k), code_phase=float(rng.uniform(0, 511)),
               doppler=float(rng.uniform(-5000, 5000)), cn0=44.0, data_bits=1) for k in glo]
    if_gps = gc.ifgen(10 * N, sg, fs=FS, seed=0x5EED0005)
    if_glo = gc.ifgen(10 * N, sl, fs=FS, if_glo=1.0e6, seed=0x5EED0006)
    fsky = FullSky(FS, 10, N_BINS, rank=dist.rank, world=dist.world, device=dev)
    fsky.load(if_gps, if_glo)
    for _ in range(warmup):
        fsky.run()
    fsky.sync()
    dist.barrier()
    gc.dev_synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        fsky.run()
    fsky.sync()
    gc.dev_synchronize(dev)
    t1 = time.perf_counter()
    dist.barrier()
    dt = dist.max(t1 - t0)
    allres = dist.gather(fsky.results())
    found = None
    if dist.rank == 0:
        res = merge(allres)
        found = sum(1 for p in gps if res[int(p) - 1][3]["metric"] > 2.5) + \
            sum(1 for k in glo if res[32 + int(k) + 7][3]["metric"] > 2.5)
    proj = None
    # (BENCH_FULLSKY_PROJECTION=0: the per-section PMC pass, whose per-launch
    # averages would otherwise mix the shard launches of every world size)
    if dist.world == 1 and os.environ.get("BENCH_FULLSKY_PROJECTION", "1") != "0":
        del fsky
        proj = fullsky_shard_projection(dev, if_gps, if_glo, steps, dt / steps)
    return dict(dt=dt, steps=steps, found=found, n_planted=len(gps) + len(glo),
                cells=46 * N_BINS * N * 10, projection=proj)


def fullsky_shard_projection(dev, if_gps, if_glo, steps, t1):
    """The strong-scaling curve of config 5 measured shard by shard on one GPU: for
    world = 2, 4, 8 every rank's shard (gnsscorr/fullsky.py round-robin) is searched
    alone, one after another, and the slowest rank sets that world's search time
    (the shards share no data and need no collective, so a rank's time on its own
    GPU is its time alone on this one)."""
    from gnsscorr.fullsky import FullSky
    out = {"world_1_ms": t1 * 1e3}
    for w in (2, 4, 8):
        per = []
        for r in range(w):
            f = FullSky(FS, 10, N_BINS, rank=r, world=w, device=dev)
            f.load(if_gps, if_glo)
            f.run()
            f.sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                f.run()
            f.sync()
            per.append((time.perf_counter() - t0) / steps)
            del f
        out[f"world_{w}"] = {"max_rank_ms": max(per) * 1e3, "min_rank_ms": min(per) * 1e3,
                             "speedup": t1 / max(per), "efficiency": t1 / max(per) / w}
    return out


GLO_COH, GLO_BAND_KHZ = 5, 12.0   # GLONASS initSettings.sci: acqCohIntegration 5, acqSearchBand 12


GLO_COH_RECORDS = int(os.environ.get("BENCH_GLO_COH_RECORDS", "16"))   # searches per step


def run_glo_coherent(dist, dev, steps, warmup, records=None):
    """The GLONASS receiver's default acquisition (initSettings.sci:88-96): 14 FCH x 121 bins
    (12 kHz at 100 Hz) x 2 blocks of 5 ms coherent, resident IF, `records` consecutive
    records of one stream per step (gnsscorr_acq_set_records, as the config-2 line)."""
    records = GLO_COH_RECORDS if records is None else records
    rng = np.random.default_rng(0x5EED0009 + dist.rank)
    glo = rng.choice(np.arange(-7, 7), 4, replace=False)
    sl = [dict(system=1, fch=int(k), code_phase=float(rng.uniform(0, 511)),
               doppler=float(rng.uniform(-5000, 5000)), cn0=39.0) for k in glo]
    IF = gc.ifgen(records * 2 * GLO_COH * N, sl, fs=FS, if_glo=1.0e6, seed=0x5EED000A + dist.rank)
    nb = int(round(GLO_BAND_KHZ * 2 * GLO_COH)) + 1
    freqs, gf = [], []
    for k in range(-7, 7):                                # acquisition.sci:105-108
        c0 = 1.0e6 + k * 0.5625e6
        gf.append(np.arange(len(freqs), len(freqs) + nb))
        freqs.extend(c0 - (GLO_BAND_KHZ / 2) * 1000 + (1000 / (2 * GLO_COH)) * np.arange(nb))
    freqs, gf = np.array(freqs), np.array(gf, np.int32)
    ctx = gc.AcqCtx(FS, N, device=dev, max_freqs=len(freqs), max_blocks=2 * GLO_COH * records,
                    max_codes=1)
    ctx.set_codes(gc.sample_code(gc.st_code(), 0.511e6, FS, N)[None])   # makeStTable.sci
    ctx.set_coherent(GLO_COH)
    if records > 1:
        ctx.set_records(records)
    d_if = gc.DevBuf.from_array(IF, dev)
    d_f = gc.DevBuf.from_array(freqs, dev)
    d_gc = gc.DevBuf.from_array(np.zeros(14, np.int32), dev)
    d_gf = gc.DevBuf.from_array(gf, dev)
    d_rows = gc.DevBuf(records * 14 * nb * gc.ACQ_ROW.itemsize, dev)
    d_res = gc.DevBuf(records * 14 * gc.ACQ_RESULT.itemsize, dev)

    def step():
        ctx.search_dev(d_if.ptr, 2, len(freqs), d_f.ptr, 14, nb, d_gc.ptr, d_gf.ptr, d_rows.ptr,
                       d_res.ptr, spc=32)
    for _ in range(warmup):
        step()
    ctx.sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    dt = dist.max(time.perf_counter() - t0)
    res = d_res.download(np.uint8).view(gc.ACQ_RESULT).reshape(records, 14)
    found = int(sum(res[r][int(k) + 7]["metric"] > 2.5 for r in range(records) for k in glo))
    return dict(dt=dt, steps=steps, nb=nb, found=found, n_planted=records * len(glo),
                records=records)


GPS_SCI_FS, GPS_SCI_COH, GPS_SCI_BAND = 16.0e6, 4, 14.0   # SCI/GPS/L1/initSettings.sci:68-87


GPS_SCI_RECORDS = int(os.environ.get("BENCH_GPS_SCI_RECORDS", "16"))   # searches per step (as ACQ_RECORDS)


def run_gps_scilab(dist, dev, steps, warmup, records=None):
    """The Scilab GPS receiver's own default acquisition (initSettings.sci:68-87):
    fs 16 MHz (samplesPerCode 16000: the 40 x 40 x 10 fp64 plan), 32 PRN x 113 bins
    (14 kHz at 125 Hz) x 2 blocks of 4 ms coherent, resident IF, `records` consecutive
    records of one stream per step (gnsscorr_acq_set_records, as the config-2 line;
    acquisition.sci:46-192 per record; parity in tests/test_acq_16m_gpu.py)."""
    records = GPS_SCI_RECORDS if records is None else records
    fs, n = GPS_SCI_FS, int(round(GPS_SCI_FS / 1000.0))
    rng = np.random.default_rng(0x5EED0040 + dist.rank)
    planted = rng.choice(np.arange(1, 33), 6, replace=False)
    sigs = [dict(system=0, prn=int(p), code_phase=float(rng.uniform(0, 1023)),
                 doppler=float(rng.uniform(-5000, 5000)), cn0=44.0, data_bits=1) for p in planted]
    IF = gc.ifgen(records * 2 * GPS_SCI_COH * n, sigs, fs=fs, seed=0x5EED0041 + dist.rank)
    nb = int(round(GPS_SCI_BAND * 2 * GPS_SCI_COH)) + 1         # acquisition.sci:101-104
    freqs = 2.42e6 - (GPS_SCI_BAND / 2) * 1000 + (1000 / (2 * GPS_SCI_COH)) * np.arange(nb)
    codes = np.stack([gc.sample_code(gc.ca_code(p), 1.023e6, fs, n) for p in range(1, 33)])
    ctx = gc.AcqCtx(fs, n, device=dev, max_freqs=nb, max_blocks=2 * GPS_SCI_COH * records,
                    max_codes=32)
    ctx.set_codes(codes)
    ctx.set_coherent(GPS_SCI_COH)
    if records > 1:
        ctx.set_records(records)
    d_if = gc.DevBuf.from_array(IF, dev)
    d_f = gc.DevBuf.from_array(freqs, dev)
    d_gc = gc.DevBuf.from_array(np.arange(32, dtype=np.int32), dev)
    d_gf = gc.DevBuf.from_array(np.tile(np.arange(nb, dtype=np.int32), 32), dev)
    d_rows = gc.DevBuf(records * 32 * nb * gc.ACQ_ROW.itemsize, dev)
    d_res = gc.DevBuf(records * 32 * gc.ACQ_RESULT.itemsize, dev)

    def step():
        ctx.search_dev(d_if.ptr, 2, nb, d_f.ptr, 32, nb, d_gc.ptr, d_gf.ptr, d_rows.ptr,
                       d_res.ptr, spc=16)
    for _ in range(warmup):
        step()
    ctx.sync()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    dt = dist.max(time.perf_counter() - t0)
    res = d_res.download(np.uint8).view(gc.ACQ_RESULT).reshape(records, 32)
    found = int(sum(res[r][int(p) - 1]["metric"] > 2.5 for r in range(records) for p in planted))
    return dict(dt=dt, steps=steps, nb=nb, n=n, found=found, n_planted=records * len(planted),
                records=records)


SDR_REC, SDR_SV, SDR_ROWS, SDR_N = 64, 32, 120, 2048
SDR_CORR_CH = 4096
# doAcqStrong int-op model per (sv, row): cmulsc 8/sample, 2048-pt int16 IFFT (11 ranks x
# 1024 radix-2 butterflies x 12 ops), cmag + max 4/sample
SDR_STRONG_OPS_ROW = 2048 * 8 + 11 * 1024 * 12 + 2048 * 4
# Correlator::Accum bytes per channel-packet: its carrier-table row (2048 CPX x 4 B),
# three code-bit rows (3 x 2048 bits) and its share of the packet (16 packets / 4096 ch)
SDR_ACCUM_BYTES = 2048 * 4 + 3 * 2048 // 8 + 16 * 2048 * 4 / SDR_CORR_CH
SDR_FE_BLOCKS = 2000         # GN3S 5-ms reads per front-end launch (10 s of 4 Msps 2-bit samples)
SDR_CHAN_N, SDR_CHAN_MS = 8192, 1000   # Channel objects x 1-ms Channel::Accum calls per launch
SDR_LOOP_RX, SDR_LOOP_REP, SDR_LOOP_PK = 8, 32, 100   # closed loop: 8 receivers' streams x 12
                                                       # channels, replicated 32x; packets/launch


def run_sdr(dist, dev, steps, warmup):
    """GPS-SDR integer paths: strong acquisition (doAcqStrong, 32 sv x 120 rows per 1-ms
    buffer, SDR_REC receivers' buffers per launch) and the batched Correlator::Accum
    (SDR_CORR_CH channels x one 2048-sample packet)."""
    rng = np.random.default_rng(0x5EED0007 + dist.rank)
    bufs = rng.integers(-3, 4, (SDR_REC, SDR_N, 2)).astype(np.int16)
    acq = gc.SdrAcqCtx(38400.0, device=dev)
    d_b = gc.DevBuf.from_array(bufs, dev)
    d_sv = gc.DevBuf.from_array(np.arange(SDR_SV, dtype=np.int32), dev)
    d_r = gc.DevBuf(SDR_REC * SDR_SV * gc.SDR_RESULT.itemsize, dev)
    for _ in range(warmup):
        acq.strong_dev(d_b.ptr, SDR_REC, SDR_SV, d_sv.ptr, d_r.ptr)
    acq.sync()
    e0, e1 = gc.Event(dev), gc.Event(dev)
    dist.barrier()
    t0 = time.perf_counter()
    e0.record(acq.stream)
    for _ in range(steps):
        acq.strong_dev(d_b.ptr, SDR_REC, SDR_SV, d_sv.ptr, d_r.ptr)
    e1.record(acq.stream)
    acq.sync()
    dt_acq = dist.max(time.perf_counter() - t0)
    ms_acq = e0.elapsed_ms(e1) / steps
    # batched Accum: every channel a full packet, random bins/offsets
    corr = gc.SdrCorrCtx(device=dev)
    pk = rng.integers(-3, 4, (16, SDR_N, 2)).astype(np.int16)
    jobs = np.zeros(SDR_CORR_CH, gc.SDR_JOB)
    jobs["packet"] = np.arange(SDR_CORR_CH) % 16
    jobs["samps"] = SDR_N
    jobs["sv"] = rng.integers(0, 32, SDR_CORR_CH)
    jobs["sbin"] = rng.integers(1000, 2000, SDR_CORR_CH)
    jobs["soff"] = rng.integers(0, 2048, SDR_CORR_CH)
    jobs["cbin"] = rng.integers(0, 101, (SDR_CORR_CH, 3))
    jobs["coff"] = rng.integers(0, 2048, (SDR_CORR_CH, 3))
    d_pk = gc.DevBuf.from_array(pk, dev)
    d_j = gc.DevBuf.from_array(jobs, dev)
    d_o = gc.DevBuf(SDR_CORR_CH * gc.SDR_CORR.itemsize, dev)
    for _ in range(warmup):
        corr.accum_dev(d_pk.ptr, SDR_CORR_CH, d_j.ptr, d_o.ptr)
    corr.sync()
    dist.barrier()
    t0 = time.perf_counter()
    e0.record(corr.stream)
    for _ in range(steps):
        corr.accum_dev(d_pk.ptr, SDR_CORR_CH, d_j.ptr, d_o.ptr)
    e1.record(corr.stream)
    corr.sync()
    dt_corr = dist.max(time.perf_counter() - t0)
    ms_corr = e0.elapsed_ms(e1) / steps
    # sample front end: GN3S 2-bit packed bytes -> 2.048 Msps CPX, SDR_FE_BLOCKS x 5 ms
    fe = gc.SdrFeCtx(device=dev)
    d_fi = gc.DevBuf(SDR_FE_BLOCKS * gc.GN3S_BLOCK_IN // 4, dev)
    d_fi.fill_if2(0x5EED0008 + dist.rank)
    d_fo = gc.DevBuf(SDR_FE_BLOCKS * gc.GN3S_BLOCK_OUT * 4, dev)
    ph = 0
    for _ in range(warmup):
        ph = fe.gn3s_dev(d_fi.ptr, True, SDR_FE_BLOCKS, ph, d_fo.ptr)
    fe.sync()
    dist.barrier()
    t0 = time.perf_counter()
    e0.record(fe.stream)
    for _ in range(steps):
        ph = fe.gn3s_dev(d_fi.ptr, True, SDR_FE_BLOCKS, ph, d_fo.ptr)
    e1.record(fe.stream)
    fe.sync()
    dt_fe = dist.max(time.perf_counter() - t0)
    ms_fe = e0.elapsed_ms(e1) / steps
    # medium / weak acquisition: one receiver's full request (32 sv, +-15 kHz) per step,
    # doPrepIF (10 / 310 ms) + doAcqMedium / doAcqWeak, the 310-ms record resident in HBM
    long = rng.integers(-3, 4, (310 * SDR_N, 2)).astype(np.int16)
    d_l = gc.DevBuf.from_array(long, dev)
    mw = {}
    for kind, t, k_steps in (("medium", gc.SDR_ACQ_MEDIUM, steps), ("weak", gc.SDR_ACQ_WEAK,
                                                                   max(steps // 5, 3))):
        for _ in range(2):
            acq.prep_dev(t, d_l.ptr, 1)
            acq.search_dev(t, 1, SDR_SV, d_sv.ptr, d_r.ptr, -15000, 15000)
        acq.sync()
        dist.barrier()
        t0 = time.perf_counter()
        e0.record(acq.stream)
        for _ in range(k_steps):
            acq.prep_dev(t, d_l.ptr, 1)
            acq.search_dev(t, 1, SDR_SV, d_sv.ptr, d_r.ptr, -15000, 15000)
        e1.record(acq.stream)
        acq.sync()
        mw[kind] = dict(dt=dist.max(time.perf_counter() - t0), ms=e0.elapsed_ms(e1) / k_steps,
                        steps=k_steps)
    # Channel objects (bit lock, frame sync, parity, C/N0, loops): SDR_CHAN_N channels x
    # SDR_CHAN_MS 1-ms Channel::Accum calls per launch on synthetic navigation streams
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import sdr_nav_scenarios as nav
    corr1 = nav.correlations(SDR_CHAN_MS, nav.nav_bits(2, seed=3 + dist.rank), 7, 4000.0, 900.0,
                             seed=5 + dist.rank, q_bias=0.02)
    shift = np.arange(SDR_CHAN_N) % 20                     # different bit phases per channel
    corr = np.stack([np.roll(corr1, int(k), 0) for k in shift], 1)
    chans0 = np.zeros(SDR_CHAN_N, gc.SDR_CHANNEL)
    for k in range(SDR_CHAN_N):
        chans0[k] = gc.SdrCorrCtx.channel_start(k, k % 32, 1000 + 10 * (k % 50), 1)
    d_cc = gc.DevBuf.from_array(corr, dev)
    d_ch = gc.DevBuf.from_array(chans0, dev)
    d_last = gc.DevBuf(SDR_CHAN_N * gc.SDR_FEEDBACK.itemsize, dev)
    d_ev = gc.DevBuf(4096 * gc.SDR_SUBFRAME.itemsize, dev)
    d_ne = gc.DevBuf.from_array(np.zeros(1, np.int32), dev)
    ch_steps = max(steps // 10, 3)
    corr_ctx_k = gc.SdrCorrCtx(device=dev)
    corr_ctx_k.channel_accum_dev(SDR_CHAN_N, SDR_CHAN_MS, d_cc.ptr, d_ch.ptr, None, d_last.ptr,
                                 d_ev.ptr, 4096, d_ne.ptr)
    corr_ctx_k.sync()
    d_ch.upload(chans0)
    dist.barrier()
    t0 = time.perf_counter()
    e0.record(corr_ctx_k.stream)
    for _ in range(ch_steps):   # consecutive launches continue the same channels
        corr_ctx_k.channel_accum_dev(SDR_CHAN_N, SDR_CHAN_MS, d_cc.ptr, d_ch.ptr, None,
                                     d_last.ptr, d_ev.ptr, 4096, d_ne.ptr)
    e1.record(corr_ctx_k.stream)
    corr_ctx_k.sync()
    dt_ch = dist.max(time.perf_counter() - t0)
    ms_ch = e0.elapsed_ms(e1) / ch_steps
    loop = run_sdr_loop(dist, dev, rng)
    return dict(dt_acq=dt_acq, ms_acq=ms_acq, dt_corr=dt_corr, ms_corr=ms_corr, steps=steps,
                bufs=bufs, dt_fe=dt_fe, ms_fe=ms_fe, mw=mw, long=long, dt_ch=dt_ch, ms_ch=ms_ch,
                ch_steps=ch_steps, ch_corr=corr1, loop=loop)


def sdr_loop_scene(rng, n_pk):
    """SDR_LOOP_RX receivers' 2.048 Msps CPX streams (8 C/A signals each + noise, int16)
    and 12 channels per receiver (8 on the signals, 4 on empty codes)."""
    n = n_pk * SDR_N
    t = np.arange(n) / 2.048e6
    pk = np.zeros((n_pk, SDR_LOOP_RX, SDR_N, 2), np.int16)
    chans = []
    for r in range(SDR_LOOP_RX):
        svs = rng.choice(32, 12, replace=False)
        z = 2.0 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
        for j, sv in enumerate(svs):
            cp0, dop = float(rng.uniform(0, 1023)), float(rng.integers(-16, 17) * 250)
            if j < 8:
                chips = gc.ca_code(int(sv) + 1).astype(np.float64)
                cp = (cp0 + t * 1.023e6 * (1 + dop / 1575.42e6)) % 1023
                z += 3.0 * chips[cp.astype(np.int64)] * np.exp(2j * np.pi * (38400.0 + dop) * t)
                cs = int(round((1023 - cp0) * 2048 / 1023)) % 2048
            else:
                cs = int(rng.integers(0, 2048))
            chans.append((r, int(sv), cs, int(dop)))
        pk[:, r, :, 0] = np.clip(np.round(z.real), -127, 127).reshape(n_pk, SDR_N)
        pk[:, r, :, 1] = np.clip(np.round(z.imag), -127, 127).reshape(n_pk, SDR_N)
    return pk, chans


def run_sdr_loop(dist, dev, rng):
    """The device-resident GPS-SDR closed loop (gnsscorr_sdr_track_dev): Correlate's packet
    schedule, UpdateState, DumpAccum and Channel::Accum per dump, SDR_LOOP_PK packets per
    launch for SDR_LOOP_RX * 12 * SDR_LOOP_REP channels; consecutive launches continue the
    same channels.  Work = dumps (1-ms correlations through the whole loop) counted from
    the correlator states' dump counters of the channels still active at the end."""
    pk, chans = sdr_loop_scene(rng, 2 * SDR_LOOP_PK)
    ctx = gc.SdrCorrCtx(device=dev)
    chans = chans * SDR_LOOP_REP
    n = len(chans)
    st = np.zeros(n, gc.SDR_CHAN)
    ch = np.zeros(n, gc.SDR_CHANNEL)
    for c, (r, sv, cs, dop) in enumerate(chans):
        st[c] = ctx.init_chan(sv, cs, dop, 0.0)
        ch[c] = ctx.channel_start(c, sv, dop, 1)
    rx = np.array([c[0] for c in chans], np.int32)
    half = SDR_LOOP_PK * SDR_LOOP_RX * SDR_N * 4
    d_pk = gc.DevBuf.from_array(pk, dev)
    d_rx, d_st, d_c, d_ch = (gc.DevBuf.from_array(a, dev) for a in
                             (rx, st, np.zeros(n, gc.SDR_CORR), ch))
    d_stat = gc.DevBuf.from_array(np.zeros(n, np.int32), dev)
    d_ev = gc.DevBuf(4096 * gc.SDR_SUBFRAME.itemsize, dev)
    d_ne = gc.DevBuf.from_array(np.zeros(1, np.int32), dev)

    def launch(i):
        ctx.track_dev(d_pk.ptr + (i % 2) * half, SDR_LOOP_PK, SDR_LOOP_RX, n, d_rx.ptr,
                      d_st.ptr, d_c.ptr, d_ch.ptr, None, None, 0, None, d_stat.ptr, d_ev.ptr,
                      4096, d_ne.ptr)

    launch(0)
    ctx.sync()
    c0 = d_st.download(np.uint8).view(gc.SDR_CHAN)["count"].astype(np.int64)
    k_steps = 4
    e0, e1 = gc.Event(dev), gc.Event(dev)
    dist.barrier()
    t0 = time.perf_counter()
    e0.record(ctx.stream)
    for i in range(k_steps):
        launch(i + 1)
    e1.record(ctx.stream)
    ctx.sync()
    dt = dist.max(time.perf_counter() - t0)
    ms = e0.elapsed_ms(e1) / k_steps
    s1 = d_st.download(np.uint8).view(gc.SDR_CHAN)
    live = s1["active"] != 0
    dumps = int((s1["count"].astype(np.int64) - c0)[live].sum())
    status = d_stat.download(np.int32)
    return dict(dt=dt, ms=ms, steps=k_steps, channels=n, live=int(live.sum()),
                dumps=dumps, stopped=int((status != 0).sum()), pk=pk, chans=chans[:12])


def cpu_baseline_sdr(bufs, budget_s=5.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sdr_oracle
    o = sdr_oracle.OracleSDR()
    codes = o.prn_codes()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        o.acq_strong(bufs[n % len(bufs)], codes, list(range(SDR_SV)))
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n * SDR_SV * SDR_ROWS * SDR_N / dt, unit="cells/s", cores=1, kind="port",
                sample=f"{n} doAcqStrong searches (32 sv x 120 rows) of the scalar C restatement "
                       f"(oracle/sdr_acq.c, bit-exact with the reference -DNO_SIMD build), "
                       f"{dt:.1f} s")


def cpu_baseline_sdr_accum(budget_s=3.0):
    """Correlator::Accum on the host: the scalar C restatement (oracle/sdr_corr.c, sdrc_accum:
    cmulsc >> 14 + E/P/L prn_accum_new) over one 2048-sample packet per call."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes
    import sdr_oracle
    o = sdr_oracle.OracleSdrCorr()
    rng = np.random.default_rng(0x5EED0006)
    data = rng.integers(-512, 512, (2048, 2), dtype=np.int16)
    res = np.zeros(1, sdr_oracle.CORR)
    sine = o.carrier.reshape(-1, 2)[: 2048]
    rows = [np.ascontiguousarray(o.code.reshape(-1)[k * sdr_oracle.ROW:k * sdr_oracle.ROW + 2048])
            for k in range(3)]
    args = [ctypes.c_void_p(a.ctypes.data) for a in (data, sine, rows[0], rows[1], rows[2])]
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        o.L.sdrc_accum(*args, 2048, 0, ctypes.c_void_p(res.ctypes.data))
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit="channel-ms/s", cores=1, kind="port",
                sample=f"{n} Accum calls of 2048 samples (scalar C restatement oracle/sdr_corr.c, "
                       f"pinned to the reference primitives; includes ctypes call overhead), "
                       f"{dt:.1f} s")


SDR_MW_ROWS = {"medium": 4 * 31, "weak": 8 * 30}      # +-15 kHz (acquisition.cpp:324, :452)
SDR_MW_PASSES = {"medium": 1, "weak": 15}
# integer-op model per row pass: ten cmulsc'd 2048-sample rows (8 ops/sample),
# ten 2048-point int16 IFFTs (11 x 1024 butterflies x 12 ops), 2048 columns x 10 post-DFT
# bins x (10 complex MACs = 80 ops + |.|^2 3 + accumulate/compare 1)
SDR_MW_OPS_PASS = 10 * SDR_N * 8 + 10 * 11 * 1024 * 12 + SDR_N * 10 * 84


def cpu_baseline_sdr_loop(loop, budget_s=4.0):
    """Correlator::Correlate on the host, scalar (oracle/sdr_corr.c: schedule, Accum,
    UpdateState, DumpAccum) with its deterministic loop callback standing in for
    Channel::Accum, over receiver 0's 12 channels, packet after packet."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sdr_oracle
    o = sdr_oracle.OracleSdrCorr()
    chans = loop["chans"]
    st = np.zeros(len(chans), sdr_oracle.CHAN)
    for c, (r, sv, cs, dop) in enumerate(chans):
        st[c] = o.init_chan(sv, cs, dop, 0.0)
    corr = np.zeros(len(chans), sdr_oracle.CORR)
    pk = loop["pk"]
    k = [0]

    def run(calls):
        c0 = st["count"].astype(np.int64)
        for _ in range(calls):
            o.correlate(pk[k[0] % len(pk), 0], st, corr)
            k[0] += 1
        return int((st["count"].astype(np.int64) - c0)[st["active"] != 0].sum())

    dumps, dt, n = _timed(run, budget_s)
    return dict(value=dumps / dt, unit="channel-ms/s", cores=1, kind="port",
                sample=f"{n} packets x {len(chans)} channels of the scalar C restatement "
                       "(oracle/sdr_corr.c: Correlate + Accum + UpdateState + DumpAccum; "
                       "deterministic loop callback instead of Channel::Accum)")


def cpu_baseline_sdr_mw(long, kind, budget_s=4.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sdr_oracle
    o = sdr_oracle.OracleSDR()
    codes = o.prn_codes()
    rows = o.new_rows()
    o.prep_rows(rows, long, 310 if kind == "weak" else 10)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:   # one sv x one 1-kHz step (4 / 8 rows) per call
        lo = -15000 + 1000 * (n % 30)
        o.acq_search(kind, rows, codes, [n % SDR_SV], lo, lo + (0 if kind == "medium" else 1000))
        n += 1
    dt = time.perf_counter() - t0
    rows_done = n * (4 if kind == "medium" else 8)
    return dict(value=rows_done * 10 * SDR_N / dt, unit="cells/s", cores=1, kind="port",
                sample=f"{rows_done} doAcq{kind.capitalize()} rows (one sv x one 1-kHz step per "
                       f"call) of the scalar C restatement (oracle/sdr_acq.c, bit-exact with the "
                       f"reference -DNO_SIMD primitives), {dt:.1f} s")


def cpu_baseline_sdr_channel(corr, budget_s=3.0):
    """The reference Channel class itself (oracle/_ref, when it travelled with the tree)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sdr_oracle
    if not sdr_oracle.have_ref_chan():
        return None
    r = sdr_oracle.RefSdrChannel(0)
    r.start(0, 1000, 1)
    n, t0 = 0, time.perf_counter()
    row = np.zeros(6, np.int32)
    fb = np.zeros(1, r.FB)
    while time.perf_counter() - t0 < budget_s:
        row[:] = corr[n % len(corr)]
        r.L.ref_chan_accum(r.h, row.ctypes.data, fb.ctypes.data)
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit="channel-ms/s", cores=1, kind="reference",
                sample=f"{n} Channel::Accum calls of the reference Channel class built from "
                       f"objects/channel.cpp (oracle/_ref/libsdr_chan_ref.so; includes ctypes "
                       f"call overhead), {dt:.1f} s")


def cpu_baseline_sgt(budget_s=6.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import sgt_oracle
    s = sgt_oracle.settings(1, samplingFreq=SGT_FS)
    n_ms = 40
    IF = np.random.default_rng(3).choice(np.array([-3, -1, 1, 3], np.int8),
                                         size=2 * int(SGT_FS * (n_ms + 2) / 1000))
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        for k in range(-7, 7):
            n += len(sgt_oracle.track(IF, s, k, 100, 1e6 + 0.5625e6 * k, n_ms)["I_P"])
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit="channel-ms/s", cores=1, kind="port",
                sample=f"{n} channel-epochs of the fp64 numpy tracking.sci restatement "
                       f"(oracle/sgt_oracle.py, 14 FCH x {n_ms} ms), {dt:.1f} s")


def cpu_baseline_acq(meta, budget_s=12.0):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import acq_oracle
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    workers = max(1, min(16, aff or 1))
    gf1 = np.tile(np.arange(N_BINS), (N_PRN, 1))
    t0 = time.perf_counter()
    acq_oracle.acquire_batched(meta["IF"], FS, meta["codes"], meta["freqs"], gf1, workers=1)
    one = CELLS_PER_SEARCH / (time.perf_counter() - t0)
    gf = np.tile(np.arange(N_BINS), (N_PRN, 1))
    n, t0 = 0, time.perf_counter()
    while True:
        acq_oracle.acquire_batched(meta["IF"], FS, meta["codes"], meta["freqs"], gf,
                                   workers=workers)
        n += 1
        if time.perf_counter() - t0 > budget_s or n >= 50:
            break
    dt = time.perf_counter() - t0
    return dict(value=n * CELLS_PER_SEARCH / dt, unit="cells/s", cores=workers, kind="port",
                sample=f"{n} full 32x41 searches (fp64 numpy/scipy pocketfft restatement of "
                       f"acquisition.sci, oracle/acq_oracle.py), {dt:.1f} s",
                port_1core=dict(value=one, cores=1, sample="1 full 32x41 search, 1 worker"),
                host=host_info())


def cpu_baseline_fullsky(budget_s=8.0):
    """Config 5 on the host: the fp64 acquisition.sci restatement in non-coherent
    mode (oracle/acq_oracle.py acquire, numpy pocketfft, one core) over GPS
    groups of the same shape (41 bins x 16368 x 10 ms), as many as fit the budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import acq_oracle
    IF = gc.ifgen(10 * N, [dict(system=0, prn=3, code_phase=100.0, doppler=1000.0, cn0=45.0)],
                  fs=FS, seed=0x5EED000D)
    freqs = 2.42e6 + 500.0 * (np.arange(N_BINS) - (N_BINS - 1) / 2.0)
    n, t0 = 0, time.perf_counter()
    while True:
        code = acq_oracle.make_ca_table_row(n % 32 + 1, FS)[None]
        acq_oracle.acquire(IF, FS, code, freqs, np.arange(N_BINS)[None], n_blocks=10,
                           noncoherent=True)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return dict(value=n * N_BINS * N * 10 / dt, unit="cell-ms/s", cores=1, kind="port",
                sample=f"{n} GPS groups x {N_BINS} bins x 10 ms non-coherent (fp64 numpy "
                       f"restatement of acquisition.sci, oracle/acq_oracle.py), {dt:.1f} s")


def cpu_baseline_glo_coh(budget_s=6.0):
    """GLONASS default acquisition on the host: the fp64 restatement with the literal
    5-ms (81 840-point) coherent transforms (oracle/acq_oracle.py, one core), one FCH
    group of 121 bins at a time, as many as fit the budget."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import acq_oracle
    nb = int(round(GLO_BAND_KHZ * 2 * GLO_COH)) + 1
    IF = gc.ifgen(2 * GLO_COH * N, [dict(system=1, fch=0, code_phase=100.0, doppler=500.0,
                                         cn0=44.0)], fs=FS, if_glo=1.0e6, seed=0x5EED000E)
    code = acq_oracle.make_st_table_row(FS)[None]
    n, t0 = 0, time.perf_counter()
    while True:
        k = n % 14 - 7
        freqs = 1.0e6 + k * 0.5625e6 - (GLO_BAND_KHZ / 2) * 1000 + (1000 / (2 * GLO_COH)) * \
            np.arange(nb)
        acq_oracle.acquire(IF, FS, code, freqs, np.arange(nb)[None], group_code=np.zeros(1, int),
                           spc=32, coh=GLO_COH)
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return dict(value=n * nb * N / dt, unit="cells/s", cores=1, kind="port",
                sample=f"{n} FCH groups x {nb} bins x 2 blocks of {GLO_COH} ms coherent (fp64 "
                       f"numpy restatement with 81 840-point transforms, oracle/acq_oracle.py), "
                       f"{dt:.1f} s")


def host_info():
    """The host cores the CPU baselines ran on (nproc, affinity, model)."""
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return dict(nproc=os.cpu_count(), affinity=aff, cpu_model=model)


def _timed(fn, budget_s):
    """Run fn(calls) -> work with calls grown until one run takes >= budget/4,
    then once more sized to the budget; returns (work, seconds, calls)."""
    calls = 20
    while True:
        t0 = time.perf_counter()
        fn(calls)
        probe = time.perf_counter() - t0
        if probe >= budget_s / 4 or calls >= 1 << 20:
            break
        calls *= 4
    calls = max(calls, int(calls * budget_s / max(probe, 1e-3)))
    t0 = time.perf_counter()
    work = fn(calls)
    return work, time.perf_counter() - t0, calls


def cpu_baseline_track(budget_s=6.0):
    """BASELINE config 3 CPU path: the REFERENCE Sim_GP2021_int (correlator.c built
    from /root/reference into oracle/_ref/libosg_ref.so) on one core -- the
    reference keeps its state in globals, one instance per process -- beside our
    C port (oracle/osg_corr.c) on one core and on all cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes as C
    import osg_oracle
    if not os.path.exists(osg_oracle.ORACLE_SO):
        return None
    IF = np.random.default_rng(1).choice(np.array([-3, -1, 1, 3], np.int8),
                                         size=16 * 32 * TRACK_NS * 2)
    o = osg_oracle.OracleOSG()
    out = {}
    threads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                         else os.cpu_count() or 1))
    for tag, th, ninst in (("port_1core", 1, 1), ("port_all_cores", threads, threads)):
        w, dt, calls = _timed(lambda c: o.L.osgo_bench(ninst, TRACK_CH, IF.ctypes.data, TRACK_NS,
                                                       c, 32, 31750430, 6710886, th), budget_s)
        out[tag] = dict(value=w / TRACK_NS / dt, cores=th,
                        sample=f"{ninst} receivers x {TRACK_CH} ch x {calls} 1-ms calls, {dt:.1f} s")
    ref = None
    if osg_oracle.have_ref():
        L = C.CDLL(osg_oracle.REF_SO)
        L.ref_bench.restype = C.c_double
        L.ref_bench.argtypes = [C.c_void_p, C.c_long, C.c_int, C.c_int, C.c_long, C.c_long]
        w, dt, calls = _timed(lambda c: L.ref_bench(IF.ctypes.data, TRACK_NS, c, 32, 31750430,
                                                    6710886), budget_s)
        ref = dict(value=w / TRACK_NS / dt, unit="channel-ms/s", cores=1, kind="reference",
                   sample=f"12 ch x {calls} 1-ms calls of the reference Sim_GP2021_int "
                          f"(correlator.c built from /root/reference, oracle/_ref/libosg_ref.so), "
                          f"{dt:.1f} s")
    base = ref or dict(value=out["port_all_cores"]["value"], unit="channel-ms/s",
                       cores=out["port_all_cores"]["cores"], kind="port",
                       sample="reference build absent: " + out["port_all_cores"]["sample"])
    base.update(out)
    base["host"] = host_info()
    return base


def acq_alg_bytes(records):
    """Algorithmic HBM bytes of one config-2 correlation launch: every code spectrum
    (32 rows) and class spectrum (2 classes x 2 blocks per record) read once, fp64
    complex (16 B per element), plus the per-(row, block) statistics written."""
    return (N_PRN + 4 * records) * N * 16 + records * N_PRN * N_BINS * N_BLK * 48


def pmc_executed_flop(kernel):
    """fp64 flops the kernel executes per config-2 record (SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes
    / records per launch of that pass) from the committed PMC pass over the config-2 section
    (profiles/pmc_fp64_mix.json), if any."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_fp64_mix.json")))
        return d[kernel]["SQ_INSTS_VALU_FLOPS_FP64"] * 64 / d["_records_per_launch"]
    except (OSError, ValueError, KeyError):
        return None


def pmc_run_bytes(section):
    """HBM bytes of one whole run of a bench section (every per-run kernel), from the
    committed per-section rocprofv3 --pmc pass (tools/pmc_summary.py --runs), if any."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
        return d[f"{section}/_run"]["hbm_bytes_per_run"]
    except (OSError, ValueError, KeyError):
        return None


def hbm_fields(traffic_bytes, seconds):
    """rocprof HBM bytes (PMC) over the measured time, against the 8 TB/s peak."""
    if traffic_bytes is None or not seconds:
        return {"hbm_GBs": None, "hbm_frac": None}
    gbs = traffic_bytes / seconds / 1e9
    return {"hbm_GBs": gbs, "hbm_frac": gbs / PEAK_HBM_GBS}


def pmc_section_bytes(section, prefix):
    """HBM bytes per launch of the kernel instance whose name starts with `prefix`
    in a per-section rocprofv3 --pmc pass (profiles/pmc_traffic.json "section/kernel",
    tools/gpu_round.sh), or None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (OSError, ValueError):
        return None
    keys = sorted(k for k in d if k.startswith(f"{section}/{prefix}"))
    return d[keys[0]]["hbm_bytes_per_launch"] if keys else None


def pmc_hbm(section, prefix, seconds):
    """{traffic, hbm_GBs, hbm_frac}: a kernel's rocprof HBM bytes per launch (its
    section's own pass) over its measured launch time, against the 8 TB/s peak."""
    b = pmc_section_bytes(section, prefix)
    return {"traffic": b, "traffic_source": f"profiles/pmc_traffic.json {section}/{prefix}*",
            **hbm_fields(b, seconds)}


def pmc_traffic(kernel, section=None):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary, if any:
    the pass over that bench section alone ("section/kernel") when recorded,
    else the whole-bench pass (an average over every section using the kernel)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
        if section and f"{section}/{kernel}" in d:
            return d[f"{section}/{kernel}"]["hbm_bytes_per_launch"]
        return d.get(kernel, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` run without torch.distributed.run: start N child
    processes of this script, one rank per GPU, with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, and wait for them.  The parent never loads
    libgnsscorr.so or touches a GPU (children are started, not exec'd).  Rank 0
    prints the JSON line (stdout is inherited).  If a rank fails, the others are
    stopped (they would wait at the rank barrier forever); the exit code is the
    first non-zero one."""
    import subprocess
    port = int(os.environ.get("MASTER_PORT", "0")) or _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   GNSSCORR_GROUP_KEY=f"{port}-{os.getpid()}")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r and not rc:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


# Order of the sections in the printed line: the driver keeps the TAIL of stdout,
# so the lines most worth reading (tracking, GLONASS tracking, full-sky shard
# projection) come last.  The headline keys come first (the contract's keys).
SECTION_ORDER = ("sdr_acquisition", "sdr_acquisition_medium", "sdr_acquisition_weak",
                 "sdr_tracking", "sdr_channel", "sdr_closed_loop", "sdr_frontend",
                 "acquisition_f32", "acquisition_generic", "gps_acquisition_scilab",
                 "glonass_acquisition_5ms",
                 "executed_fp64", "single_search", "ranks", "fullsky", "glonass_tracking",
                 "tracking")
# descriptive strings moved out of the printed line into the detail file (DESIGN.md 6
# describes every section's workload)
DETAIL_KEYS = ("config", "note", "sample", "timing", "traffic_source", "source", "host",
               "port_1core", "port_all_cores", "metric", "peak", "hbm_algorithmic_frac",
               "int_ops_frac", "flop_per_launch", "cells_per_launch", "p50_us", "max_us", "steps",
               "config4_realtime_factor", "min_rank_ms", "efficiency", "p99_ms", "found")


def _round(x, sig=4):
    if isinstance(x, bool) or not isinstance(x, float):
        return x
    return float(f"{x:.{sig}g}")


def _round_all(d, sig):
    if isinstance(d, dict):
        return {k: _round_all(v, sig) for k, v in d.items()}
    return _round(d, sig)


def compact(d, key=None):
    """A section without its descriptive strings, floats to 4 significant digits,
    units without their parenthesised model notes; a section's cpu_baseline keeps
    value, cores and kind."""
    if isinstance(d, dict):
        if key == "cpu_baseline":
            return {k: _round(v) for k, v in d.items() if k in ("value", "cores", "kind")}
        return {k: compact(v, k) for k, v in d.items() if k not in DETAIL_KEYS}
    if isinstance(d, list):
        return [compact(v) for v in d]
    if isinstance(d, str) and key in ("unit", "bound"):
        return d.split(" (")[0]
    return _round(d)


def result_line(out):
    """The one printed JSON line: the contract's headline keys as assembled (the
    workload string shortened), then every section compacted, in SECTION_ORDER."""
    head = {k: v for k, v in out.items() if k not in SECTION_ORDER}
    if isinstance(head.get("cpu_baseline"), dict):
        head["cpu_baseline"] = {k: v for k, v in head["cpu_baseline"].items()
                                if k in ("value", "unit", "cores", "kind", "sample")}
    line = {k: (_round_all(v, 5) if isinstance(v, dict) else v) for k, v in head.items()}
    # the workload string names the shape; its numbers, and the roofline's algorithmic
    # bytes, stay in the detail file (the driver keeps only the tail of stdout)
    if isinstance(line.get("config"), dict):
        line["config"] = {k: v for k, v in line["config"].items()
                          if k not in ("prns", "bins", "blocks", "samples_per_code", "cells_per_search")}
    if isinstance(line.get("roofline"), dict):
        line["roofline"].pop("hbm_algorithmic_bytes_per_launch", None)
    for k in SECTION_ORDER:
        if k in out:
            line[k] = compact(out[k])
            if k not in ("tracking", "glonass_tracking", "fullsky") and \
                    isinstance(line[k], dict) and isinstance(line[k].get("roofline"), dict):
                line[k]["roofline"].pop("kernel", None)   # named in DESIGN.md 6
    if "ranks" in line:   # every rank's device and PCI id; rank 0's runtime path, and the
        rk = out["ranks"]  # most HIP runtimes any rank maps (1: only libgnsscorr's)
        hr = [r["hip_runtime"] if isinstance(r["hip_runtime"], dict)
              else {"bound": r["hip_runtime"], "mapped": [r["hip_runtime"]]} for r in rk]
        line["ranks"] = {"device": [r["device"] for r in rk],
                         "pci": [r["pci_bus_id"] for r in rk],
                         "hip_runtime": hr[0]["bound"],
                         "runtimes_mapped_max": max(len(h["mapped"]) for h in hr)}
    g = line.get("glonass_tracking", {}).get("at_16368ksps")
    if g:   # the same line at the other rate: its rate, latency and kernel time
        line["glonass_tracking"]["at_16368ksps"] = {
            "value": g.get("value"), "config4_ms_per_epoch_14ch": g.get("config4_ms_per_epoch_14ch"),
            "frac": g.get("roofline", {}).get("frac"),
            "kernel_ms_per_launch": g.get("roofline", {}).get("kernel_ms_per_launch")}
    t = line.get("tracking", {})
    for sub in list(t.get("layouts", {}).values()) + [t.get("closed_loop", {})]:
        for k in ("unit", "calls_per_launch", "realtime_channels_per_gpu", "kernel_ms_per_launch"):
            sub.pop(k, None)   # = the tracking line's unit, TRACK_CPL and TRACK_CPL x per call
    for sub in t.get("layouts", {}).values():
        sub.get("roofline", {}).pop("kernel", None)   # packed layouts: <true, false>
    for sub in t.get("pcie_inclusive", {}).values():
        sub.pop("unit", None)
    return line


def write_detail(out):
    """The full result (every description, baseline sample and host field) to
    gpurun_out/bench_detail.json; best effort."""
    try:
        d = os.path.join(ROOT, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "bench_detail.json"), "w") as f:
            json.dump(out, f, indent=1)
    except OSError:
        pass


def stub_main(a):
    """BENCH_STUB=1 (CPU test of the launcher): every rank joins the host group,
    meets at the barrier and rank 0 prints n_gpus and the gathered ranks; no
    library, no GPU."""
    dist = Dist(load_lib=False)
    dist.barrier()
    info = dist.gather(dict(rank=dist.rank, local_rank=dist.local, pid=os.getpid(),
                            torch_loaded="torch" in sys.modules))
    t = dist.max(float(dist.rank))
    if dist.rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": dist.world, "steps": a.steps,
                          "warmup": a.warmup, "ranks": info, "max_rank": t}))
    dist.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--skip-track", action="store_true")
    a = ap.parse_args()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no external launcher: one child process per rank, before any HIP call
        raise SystemExit(launch_ranks(a.gpus, sys.argv[1:]))
    if os.environ.get("BENCH_STUB") == "1":
        return stub_main(a)
    gc.lib()           # the library binds its HIP runtime first (see Dist)
    dist = Dist()
    n_dev = gc.device_count()
    if n_dev < 1:
        raise SystemExit("bench.py: no HIP device visible")
    dev = dist.local % n_dev     # one rank per GPU; wraps only when rehearsing on fewer GPUs

    acq = run_acq(dist, dev, a.steps, a.warmup, gc.ACQ_F64)
    # one search alone per launch: the cold-start latency north_star asks for (< 1 ms wall)
    acq1 = run_acq(dist, dev, max(a.steps, 20), a.warmup, gc.ACQ_F64, records=1)
    acq32 = None if a.skip_track else run_acq(dist, dev, a.steps, a.warmup, gc.ACQ_F32)
    rank_info = dist.gather(dict(rank=dist.rank, device=dev, pci_bus_id=gc.pci_bus_id(dev),
                                 hip_runtime=gc.hip_runtime()))
    trk = None if a.skip_track else run_track(dist, dev, max(a.steps, 20), a.warmup)
    tio = None if a.skip_track else run_track_io(dist, dev, max(a.steps, 20), a.warmup)
    sgt = None if a.skip_track else run_sgt(dist, dev, max(a.steps, 20), a.warmup)
    sgt_c4 = None if a.skip_track else run_sgt(dist, dev, max(a.steps, 20), a.warmup, FS)
    # (20 timed searches after 5 warmups: 5 timed after 2 read 1.44 ms against 1.37-1.39
    # in steady state, profiles/r6/fullsky_generic_steps_r7o.log)
    sky = None if a.skip_track else run_fullsky(dist, dev, max(a.steps, 10), 5)
    sdr = None if a.skip_track else run_sdr(dist, dev, max(a.steps // 2, 10), 2)
    gco = None if a.skip_track else run_glo_coherent(dist, dev, max(a.steps, 10), 5)
    # (20 timed searches after 5 warmups: 10 timed after 3 read 0.99-1.00 ms against
    # 0.94-0.95 at 20, profiles/r6/fullsky_generic_steps_r7o.log)
    gen = None if a.skip_track else run_acq_generic(dist, dev, max(a.steps, 10), 5)
    gsc = None if a.skip_track else run_gps_scilab(dist, dev, max(a.steps, 10), 5)

    if dist.rank == 0:
        W = dist.world
        R = acq["records"]
        cells = CELLS_PER_SEARCH * a.steps * W * R
        value = cells / acq["dt"]
        flop_launch = N_PRN * N_BINS * N_BLK * N * FLOP_PER_CELL_BLOCK * R
        achieved = flop_launch / (acq["corr_ms"] * 1e-3) / 1e12
        out = {
            "metric": METRIC, "value": value, "unit": "cells/s", "n_gpus": W,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": acq["dt"] / a.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (deterministic 2-bit IQ with 8 planted GPS signals per rank)",
            "config": {"workload": "BASELINE config 2: 32-PRN x 41-bin cold-start acquisition, "
                                   "1 ms coherent, 2 blocks (acquisition.sci), 16.368 Msps, "
                                   f"fp64; {R} 2-ms records per step in one launch; code "
                                   "spectra outside the steps (inside: single_search)",
                       "code_spectra_ms": acq["meta"]["set_codes_ms"],
                       "prns": N_PRN, "bins": N_BINS, "blocks": N_BLK, "samples_per_code": N,
                       "cells_per_search": CELLS_PER_SEARCH, "records_per_step": R,
                       "parallelism": f"weak: {R} searches per GPU per step x {W} GPUs"},
            "roofline": {"bound": "valu", "kernel": ACQ64_KERNEL, "achieved": achieved,
                         "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s (fp64)",
                         "frac": achieved / PEAK_FP64_TFLOPS,
                         "traffic": pmc_traffic(ACQ64_KERNEL, "acq"),
                         "kernel_ms_per_launch": acq["corr_ms"],
                         "flop_per_launch": flop_launch,
                         # rocprof HBM bytes of this kernel per launch / its measured duration
                         **hbm_fields(pmc_traffic(ACQ64_KERNEL, "acq"), acq["corr_ms"] * 1e-3),
                         "hbm_algorithmic_bytes_per_launch": acq_alg_bytes(R)},
            "ms_per_search": acq["dt"] / a.steps / R * 1e3,
            "single_search": {"ms_per_search": acq1["dt"] / max(a.steps, 20) * 1e3,
                              "corr_kernel_ms": acq1["corr_ms"],
                              "with_codes": acq1["with_codes"],
                              "note": "one 2-ms record per launch (records_per_step = 1): the "
                                      "wall time of one complete cold-start search, "
                                      "resident IF; with_codes: the 32 replicas generated on the "
                                      "device and transformed inside each search "
                                      "(acquisition.sci:91-95), host sync per search, warm "
                                      "context"},
            # the prime-factor transform executes more fp64 flops than the radix-2 model
            # counts: its executed rate against the same peak (PMC, committed pass)
            "executed_fp64": (lambda f: None if f is None else {
                "flop_per_launch": f * R, "tflops": f * R / (acq["corr_ms"] * 1e-3) / 1e12,
                "frac": f * R / (acq["corr_ms"] * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                "source": "profiles/pmc_fp64_mix.json (SQ_INSTS_VALU_FLOPS_FP64 x 64, "
                          "per record x records per launch)"})(pmc_executed_flop(ACQ64_KERNEL)),
            "planted_found": f"{acq['found']}/{acq['n_planted']}",
            "ranks": rank_info,
        }
        if acq32:
            cells = CELLS_PER_SEARCH * a.steps * W
            a32 = flop_launch / R / (acq32["corr_ms"] * 1e-3) / 1e12
            out["acquisition_f32"] = {
                "metric": "acquisition cells/sec (config 2, single-precision fast path)",
                "value": cells / acq32["dt"], "unit": "cells/s", "dtype": "f32",
                "ms_per_step": acq32["dt"] / a.steps * 1e3,
                "note": "rows within 2e-5 of the row max of fp64 (tests/test_acq_gpu.py[f32]); "
                        "not the reference's precision",
                "roofline": {"bound": "valu", "kernel": "acq_corr_pipe_kernel", "achieved": a32,
                             "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s (fp32)",
                             "frac": a32 / PEAK_FP32_TFLOPS,
                             "traffic": pmc_traffic("acq_corr_pipe_kernel"),
                             "kernel_ms_per_launch": acq32["corr_ms"]},
                "planted_found": f"{acq32['found']}/{acq32['n_planted']}",
            }
        if gen:
            out["acquisition_generic"] = {
                "metric": "acquisition cells/sec (config-2 search at a rate without a compiled "
                          "plan: fp64 generic engine)",
                "value": N_PRN * N_BINS * gen["n"] * gen["steps"] * gen["records"] * W / gen["dt"],
                "unit": "cells/s", "dtype": "f64",
                "ms_per_search": gen["dt"] / (gen["steps"] * gen["records"]) * 1e3,
                "records_per_step": gen["records"],
                # rocprof HBM bytes of one whole step (every per-step kernel, PMC pass of
                # this section) over its time
                "roofline": {"bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
                             "traffic_per_search": (pmc_run_bytes("acq_generic") or 0) / gen["records"] or None,
                             **hbm_fields(pmc_run_bytes("acq_generic"), gen["dt"] / gen["steps"])},
                "config": f"fs = {gen['fs'] / 1e6:.3f} Msps (N = {gen['n']}): 32 PRN x 41 bins x "
                          "2 blocks per record, every length-N DFT as a four-step 112 x 341 "
                          "plan (two LDS passes, product fused into the first, |.|^2 and "
                          "per-column top-2 row statistics into the second)",
                "planted_found": f"{gen['found']}/{gen['n_planted']}",
            }
        if trk:
            C = trk["channels"]
            steps_t = trk["steps"]
            tvalue = C * steps_t * W / trk["dt"]
            bytes_launch = C * (2.0 * TRACK_NS / TRACK_CH + 64)
            ops_launch = C * TRACK_NS * TRACK_OPS_PER_SAMPLE
            k_s = trk["kern_ms"] * 1e-3          # per call
            L_s = k_s * TRACK_CPL                 # per launch (TRACK_CPL calls)
            out["tracking"] = {
                "metric": "1ms E/P/L correlations/sec", "value": tvalue, "unit": "channel-ms/s",
                "steps": steps_t, "channels_per_gpu": C,
                "config": f"{TRACK_RX} receivers x {TRACK_CH} GP2021 channels per GPU, own "
                          f"int8 IQ stream each, 1-ms calls (BASELINE config 3 scaled out)",
                "realtime_channels_per_gpu": C * 1.0 / trk["kern_ms"],
                "roofline": {"bound": "valu", "kernel": TRACK_KERNEL,
                             "achieved": ops_launch / k_s / 1e12, "peak": PEAK_INT_TOPS,
                             "unit": "Tops/s (int32, 20 ops/sample model)",
                             "frac": ops_launch / k_s / 1e12 / PEAK_INT_TOPS,
                             "hbm_algorithmic_GBs": bytes_launch / k_s / 1e9,
                             "hbm_algorithmic_frac": bytes_launch / k_s / 1e9 / PEAK_HBM_GBS,
                             **pmc_hbm("track", TRACK_KERNEL, L_s),
                             "calls_per_launch": TRACK_CPL,
                             "kernel_ms_per_call": trk["kern_ms"],
                             "kernel_ms_per_launch": trk["kern_ms"] * TRACK_CPL,
                             "us_per_3072_channel_ms": trk["kern_ms"] * 1e3 * 3072 / C},
                "dumps_sane": trk["dumps_ok"],
                "closed_loop": {
                    "metric": "1ms E/P/L correlations/sec with the gpsisr channel loops on the GPU",
                    "value": C * steps_t * W / trk["dt_cl"],
                    "unit": "channel-ms/s",
                    "config": f"{C} channels, 1-ms calls: per call the correlator "
                              f"({TRACK_KERNEL}) and then osg_isr_kernel, every channel's gpsisr "
                              "step (acquisition / confirm / pull-in / tracking state machine, 64 "
                              "channels per wave), NCO words fed back on the device, no host "
                              "round trip (GNSSCORR_OSG_FUSED=1: both in one launch of "
                              f"{TRACK_KERNEL_CL} per {TRACK_CPL} calls, 6 % slower)",
                    "ms_per_call": trk["cl_ms"],
                    "us_per_3072_channel_ms": trk["cl_ms"] * 1e3 * 3072 / C,
                    "kernel": TRACK_KERNEL + " + osg_isr_kernel", "launches_per_call": 2,
                },
            }
        if tio:
            lay = {}
            for key, desc in (("cs1_int8", "one int8 IQ stream per channel (C_s = 1)"),
                              ("cs1_packed2", "one 2-bit packed IQ stream per channel (C_s = 1)"),
                              ("rx12_packed2", f"{TRACK_RX} receivers x {TRACK_CH} channels, "
                                               "2-bit packed IQ streams")):
                r = tio[key]
                k_s = r["kern_ms"] * 1e-3
                L_s = k_s * TRACK_CPL
                lay[key] = {
                    "config": f"{r['channels']} channels, {desc}, distinct IF every call",
                    "value": r["channels"] * tio["steps"] * W / r["dt"],
                    "unit": "channel-ms/s",
                    "calls_per_launch": TRACK_CPL,
                    "kernel_ms_per_call": r["kern_ms"],
                    "kernel_ms_per_launch": r["kern_ms"] * TRACK_CPL,
                    "us_per_3072_channel_ms": r["kern_ms"] * 1e3 * 3072 / r["channels"],
                    "realtime_channels_per_gpu": r["channels"] / r["kern_ms"],
                    "roofline": {"bound": "hbm",
                                 "kernel": TRACK_KERNEL_PK if "packed" in key else TRACK_KERNEL,
                                 "achieved": r["bytes_launch"] / k_s / 1e9, "peak": PEAK_HBM_GBS,
                                 "unit": "GB/s (algorithmic: IF bytes + 64 B state/command/"
                                         "result per channel)",
                                 "frac": r["bytes_launch"] / k_s / 1e9 / PEAK_HBM_GBS,
                                 **pmc_hbm(f"trk_{key}", TRACK_KERNEL_PK if "packed" in key
                                           else TRACK_KERNEL, L_s),
                                 "int_ops_frac": r["channels"] * TRACK_NS * TRACK_OPS_PER_SAMPLE
                                 / k_s / 1e12 / PEAK_INT_TOPS},
                }
                if "ok" in r:
                    lay[key]["dumps_sane"] = r["ok"]
            out["tracking"]["layouts"] = lay
            out["tracking"]["pcie_inclusive"] = {
                k: {"config": f"gnsscorr_track from pageable host buffers: {r['channels']} "
                              f"channels on {TRACK_RX_HOST} streams, {r['h2d_bytes']} B H2D + results "
                              "D2H + stream sync per 1-ms call",
                    "value": r["channels"] / (r["mean_ms"] * 1e-3), "unit": "channel-ms/s",
                    "mean_ms_per_call": r["mean_ms"], "p99_ms_per_call": r["p99_ms"],
                    "realtime": r["p99_ms"] < 1.0}
                for k, r in (("int8", tio["host_int8"]), ("packed2", tio["host_packed2"]))}
            r = tio["sim_gp2021_12ch"]
            out["tracking"]["config3_realtime"] = {
                "config": f"BASELINE config 3 as the reference runs it: Sim_GP2021_int "
                          f"(legacy shim) for 12 channels, {r['nsamp']} samples = one 512-us "
                          f"interrupt per call (osgnss_next_step.c:150,168-184), host IF, "
                          f"{r['calls']} calls",
                "mean_us": r["mean_us"], "p50_us": r["p50_us"], "p99_us": r["p99_us"],
                "max_us": r["max_us"], "budget_us": r["budget_us"],
                "realtime": r["p99_us"] < r["budget_us"]}
        def sgt_line(sgt):
            C = sgt["channels"]
            k_s = sgt["kern_ms"] * 1e-3
            dp = C * sgt["steps"] * sgt["fs"] / 1000 * SGT_DP_PER_SAMPLE
            return {
                "metric": "1ms E/P/L correlations/sec (GLONASS L1OF float loop, tracking.sci)",
                "value": C * sgt["steps"] * W / sgt["dt"], "unit": "channel-ms/s",
                "steps": sgt["steps"], "channels_per_gpu": C,
                "config": f"BASELINE config 4 scaled out: {SGT_RX} records x 14 FCH, 511-chip ST, "
                          f"{sgt['fs'] / 1e6:g} Msps int8 IQ, fp64 NCOs + FLL/PLL/DLL on the GPU",
                "config4_ms_per_epoch_14ch": sgt["lat_ms"],
                "config4_realtime_factor": 1.0 / sgt["lat_ms"],
                "realtime_channels_per_gpu": C * sgt["steps"] / sgt["kern_ms"],
                "roofline": {"bound": "valu", "kernel": "sgt_track_kernel",
                             "achieved": dp / k_s / 1e12, "peak": PEAK_FP64_TFLOPS,
                             "unit": f"TFLOP/s (fp64, {SGT_DP_PER_SAMPLE} ops/sample model)",
                             "frac": dp / k_s / 1e12 / PEAK_FP64_TFLOPS,
                             "hbm_algorithmic_GBs": C * sgt["steps"] * sgt["fs"] / 1000 * 2 / 14
                             / k_s / 1e9,
                             # the wave-per-channel instance (>= 1024 channels); the
                             # 14-channel latency run is the <2, true, 256> one
                             **pmc_hbm("sgt", "sgt_track_kernel<2, true, 64>", k_s),
                             "kernel_ms_per_launch": sgt["kern_ms"]},
                "epochs_sane": sgt["ok"],
            }
        if sgt:
            out["glonass_tracking"] = sgt_line(sgt)
            if sgt_c4:
                # config 4 at the rate SURVEY 8(d) states (32.03 samples per ST chip)
                out["glonass_tracking"]["at_16368ksps"] = sgt_line(sgt_c4)
        if sky:
            sky_ms = sky["dt"] / sky["steps"] * 1e3
            sky_flop = sky["cells"] * FLOP_PER_CELL_BLOCK       # cell-ms x flop per cell-block
            out["fullsky"] = {
                "metric": "acquisition cell-ms/s (full-sky, 10 ms non-coherent)",
                "value": sky["cells"] * sky["steps"] / sky["dt"], "unit": "cell-ms/s",
                "scaling": "strong", "steps": sky["steps"],
                "ms_per_search": sky["dt"] / sky["steps"] * 1e3,
                "config": "BASELINE config 5: (32 GPS PRN + 14 GLONASS FCH) x 41 bins x 16368 "
                          f"x 10 ms non-coherent = {sky['cells']} cell-ms per search; groups "
                          f"sharded round-robin over {W} GPU(s), results gathered over the host group",
                "planted_found": f"{sky['found']}/{sky['n_planted']}",
                "dtype": "f64",
                "shard_projection": sky["projection"],
                "roofline": {"bound": "valu", "kernel": "acq64_corr_kernel<PlanA, NONCOHERENT>",
                             "achieved": sky_flop / (sky_ms * 1e-3) / 1e12 / W,
                             "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s (fp64, per GPU)",
                             "frac": sky_flop / (sky_ms * 1e-3) / 1e12 / W / PEAK_FP64_TFLOPS,
                             "timing": "whole search per step (forward spectra included): a "
                                       "lower bound on the correlation kernel's rate",
                             # HBM bytes of one whole search (PMC, every per-search kernel)
                             # over the search time
                             **hbm_fields(None if pmc_run_bytes("fullsky") is None else
                                          pmc_run_bytes("fullsky") / W, sky_ms * 1e-3),
                             "traffic": pmc_traffic("acq64_corr_kernel<Plan<16368, 16, 33, 31, "
                                                    "512, true>, 1, false>", "fullsky")},
            }
        if gsc:
            cells = 32 * gsc["nb"] * gsc["n"]
            fl = cells * N_BLK * (5.0 * np.log2(gsc["n"]) + 10)
            ts = gsc["dt"] / (gsc["steps"] * gsc["records"])   # seconds per search
            out["gps_acquisition_scilab"] = {
                "metric": "acquisition cells/sec (the Scilab GPS receiver's default search)",
                "value": cells * W / ts, "unit": "cells/s",
                "ms_per_search": ts * 1e3, "records_per_step": gsc["records"],
                "config": f"SCI/GPS/L1/initSettings.sci defaults: 32 PRN x {gsc['nb']} bins (14 kHz "
                          f"at 125 Hz) x 16000 code phases, 2 blocks of {GPS_SCI_COH} ms coherent, "
                          "16 Msps, fp64 (40 x 40 x 10 plan), IF resident in HBM",
                "planted_found": f"{gsc['found']}/{gsc['n_planted']}",
                "dtype": "f64",
                "roofline": {"bound": "valu", "kernel": "acq64 (whole search)",
                             "achieved": fl / ts / 1e12,
                             "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s (fp64)",
                             "frac": fl / ts / 1e12 / PEAK_FP64_TFLOPS,
                             "traffic_per_search": (pmc_run_bytes("gps_scilab") or 0) / gsc["records"] or None,
                             **hbm_fields(pmc_run_bytes("gps_scilab"), gsc["dt"] / gsc["steps"])},
            }
        if gco:
            cells = 14 * gco["nb"] * N
            tg = gco["dt"] / (gco["steps"] * gco["records"])   # seconds per search
            out["glonass_acquisition_5ms"] = {
                "metric": "acquisition cells/sec (GLONASS, 5 ms coherent, acquisition.sci)",
                "value": cells * W / tg, "unit": "cells/s",
                "ms_per_search": tg * 1e3, "records_per_step": gco["records"],
                "config": f"GLONASS initSettings.sci defaults: 14 FCH x {gco['nb']} bins (12 kHz "
                          f"at 100 Hz) x 16368 code phases, 2 blocks of {GLO_COH} ms coherent, "
                          "16.368 Msps, IF resident in HBM",
                "planted_found": f"{gco['found']}/{gco['n_planted']}",
                "dtype": "f64",
                "roofline": {"bound": "valu", "kernel": "acq64 (whole search)",
                             "achieved": cells * N_BLK * FLOP_PER_CELL_BLOCK / tg / 1e12,
                             "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s (fp64)",
                             "frac": cells * N_BLK * FLOP_PER_CELL_BLOCK / tg / 1e12 / PEAK_FP64_TFLOPS,
                             "timing": "whole search (the 5-ms folding wipe-off and forward "
                                       "spectra included)",
                             "traffic_per_search": (pmc_run_bytes("glo_coherent") or 0) / gco["records"] or None,
                             **hbm_fields(pmc_run_bytes("glo_coherent"),
                                          gco["dt"] / gco["steps"])},
            }
        if sdr:
            cells = SDR_REC * SDR_SV * SDR_ROWS * SDR_N
            ops = SDR_REC * SDR_SV * SDR_ROWS * SDR_STRONG_OPS_ROW
            out["sdr_acquisition"] = {
                "metric": "acquisition cells/sec (GPS-SDR int16 strong acquisition, bit-exact)",
                "value": cells * sdr["steps"] * W / sdr["dt_acq"], "unit": "cells/s",
                "config": f"{SDR_REC} receivers' 1-ms 2.048 Msps CPX buffers per launch x 32 sv x "
                          "120 rows (+-15 kHz: 30 x 1 kHz shifts x 4 sub-bins) x 2048 (doAcqStrong)",
                "kernel_ms_per_launch": sdr["ms_acq"],
                "cells_per_launch": cells,
                "roofline": {"bound": "valu", "kernel": "sdr_strong_kernel",
                             "achieved": ops / (sdr["ms_acq"] * 1e-3) / 1e12, "peak": PEAK_INT_TOPS,
                             "unit": "Tops/s (int32 op model, DESIGN.md)",
                             "frac": ops / (sdr["ms_acq"] * 1e-3) / 1e12 / PEAK_INT_TOPS,
                             **pmc_hbm("sdr", "sdr_strong_kernel", sdr["ms_acq"] * 1e-3)},
            }
            out["sdr_tracking"] = {
                "metric": "1ms E/P/L correlations/sec (GPS-SDR Correlator::Accum, bit-exact)",
                "value": SDR_CORR_CH * sdr["steps"] * W / sdr["dt_corr"], "unit": "channel-ms/s",
                "config": f"{SDR_CORR_CH} channels x one 2048-sample packet per launch "
                          "(wipe-off row + 3 code rows from the HBM-resident pre-sampled tables)",
                "kernel_ms_per_launch": sdr["ms_corr"],
                "roofline": {"bound": "hbm", "kernel": "sdr_accum_kernel",
                             "achieved": SDR_CORR_CH * SDR_ACCUM_BYTES / (sdr["ms_corr"] * 1e-3)
                             / 1e9, "peak": PEAK_HBM_GBS,
                             "unit": "GB/s (algorithmic: carrier row + code-bit rows + packet "
                                     "share per channel)",
                             "frac": SDR_CORR_CH * SDR_ACCUM_BYTES / (sdr["ms_corr"] * 1e-3) / 1e9
                             / PEAK_HBM_GBS,
                             **pmc_hbm("sdr", "sdr_accum_kernel", sdr["ms_corr"] * 1e-3)},
            }
            for kind, m in sdr["mw"].items():
                cells = SDR_SV * SDR_MW_ROWS[kind] * 10 * SDR_N
                ops = SDR_SV * SDR_MW_ROWS[kind] * SDR_MW_PASSES[kind] * SDR_MW_OPS_PASS
                out[f"sdr_acquisition_{kind}"] = {
                    "metric": f"acquisition cells/sec (GPS-SDR {kind} acquisition, bit-exact)",
                    "value": cells * m["steps"] * W / m["dt"], "unit": "cells/s",
                    "config": f"one receiver's full doAcq{kind.capitalize()} request per step: "
                              f"32 sv x {SDR_MW_ROWS[kind]} rows (+-15 kHz) x 10 post-DFT bins "
                              f"(25 Hz) x 2048 delays, "
                              + ("10 ms coherent" if kind == "medium" else
                                 "15 x 10 ms coherent, non-coherent sum with code-Doppler shift")
                              + " (310-ms record resident in HBM, doPrepIF included)",
                    "ms_per_search": m["ms"],
                    "roofline": {"bound": "valu", "kernel": "sdr_coh_kernel",
                                 "achieved": ops / (m["ms"] * 1e-3) / 1e12, "peak": PEAK_INT_TOPS,
                                 "unit": "Tops/s (int32 op model, DESIGN.md)",
                                 "frac": ops / (m["ms"] * 1e-3) / 1e12 / PEAK_INT_TOPS,
                                 # rocprof HBM bytes of the request's correlation launch
                                 # over the whole request time (a lower bound)
                                 **pmc_hbm("sdr", "sdr_coh_kernel<%s>" % str(kind == "weak").lower(),
                                           m["ms"] * 1e-3)},
                }
            out["sdr_channel"] = {
                "metric": "Channel::Accum calls/sec (GPS-SDR channel: bit lock, frame sync, "
                          "parity, C/N0, FLL/PLL/DLL; exact vs the reference Channel)",
                "value": SDR_CHAN_N * SDR_CHAN_MS * sdr["ch_steps"] * W / sdr["dt_ch"],
                "unit": "channel-ms/s",
                "config": f"{SDR_CHAN_N} channels x {SDR_CHAN_MS} consecutive 1-ms calls per "
                          "launch (one thread per channel), synthetic 50 bps navigation streams",
                "kernel_ms_per_launch": sdr["ms_ch"],
                "roofline": {"bound": "latency (serial per-channel chains)",
                             "kernel": "sdr_channel_kernel",
                             **pmc_hbm("sdr", "sdr_channel_kernel", sdr["ms_ch"] * 1e-3)},
            }
            lp = sdr["loop"]
            out["sdr_closed_loop"] = {
                "metric": "closed-loop channel-ms/sec (GPS-SDR Correlate schedule + UpdateState + "
                          "DumpAccum + Channel::Accum per dump, device-resident, bit-exact with "
                          "the host-scheduled loop)",
                "value": lp["dumps"] * W / lp["dt"], "unit": "channel-ms/s",
                "config": f"{lp['channels']} channels ({SDR_LOOP_RX} receivers x 12, replicated "
                          f"{SDR_LOOP_REP}x) x {SDR_LOOP_PK} consecutive 2048-sample packets per "
                          "launch (gnsscorr_sdr_track_dev, one workgroup per channel)",
                "kernel_ms_per_launch": lp["ms"],
                "channels_live_at_end": lp["live"], "channels_stopped": lp["stopped"],
                "realtime_channels_per_gpu": lp["dumps"] / lp["steps"] / lp["ms"],
                "roofline": {"bound": "latency (serial per-channel chains)",
                             "kernel": "sdr_track_kernel",
                             **pmc_hbm("sdr", "sdr_track_kernel", lp["ms"] * 1e-3)},
            }
            fe_in = SDR_FE_BLOCKS * gc.GN3S_BLOCK_IN
            fe_bytes = fe_in // 4 + SDR_FE_BLOCKS * gc.GN3S_BLOCK_OUT * 4
            out["sdr_frontend"] = {
                "metric": "input samples/sec (GPS-SDR GN3S 2-bit unpack + NCO mix + resample, "
                          "bit-exact)",
                "value": fe_in * sdr["steps"] * W / sdr["dt_fe"], "unit": "samples/s",
                "config": f"{SDR_FE_BLOCKS} x 5-ms GN3S reads (packed 2-bit, 4 Msps) -> "
                          f"{SDR_FE_BLOCKS * 5} packets of 2048 CPX per launch",
                "kernel_ms_per_launch": sdr["ms_fe"],
                "realtime_streams_per_gpu": SDR_FE_BLOCKS * 5e-3 / (sdr["ms_fe"] * 1e-3),
                "roofline": {"bound": "hbm", "achieved": fe_bytes / (sdr["ms_fe"] * 1e-3) / 1e9,
                             "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": fe_bytes / (sdr["ms_fe"] * 1e-3) / 1e9 / PEAK_HBM_GBS,
                             **pmc_hbm("sdr", "gn3s_kernel", sdr["ms_fe"] * 1e-3)},
            }
        if W == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline_acq(acq["meta"])
            if trk:
                tb = cpu_baseline_track()
                if tb:
                    out["tracking"]["cpu_baseline"] = tb
            if sgt:
                out["glonass_tracking"]["cpu_baseline"] = cpu_baseline_sgt()
            if sky:
                out["fullsky"]["cpu_baseline"] = cpu_baseline_fullsky()
            if gco:
                out["glonass_acquisition_5ms"]["cpu_baseline"] = cpu_baseline_glo_coh()
            if sdr:
                out["sdr_acquisition"]["cpu_baseline"] = cpu_baseline_sdr(sdr["bufs"])
                for kind in sdr["mw"]:
                    out[f"sdr_acquisition_{kind}"]["cpu_baseline"] = \
                        cpu_baseline_sdr_mw(sdr["long"], kind)
                out["sdr_tracking"]["cpu_baseline"] = cpu_baseline_sdr_accum()
                out["sdr_closed_loop"]["cpu_baseline"] = cpu_baseline_sdr_loop(sdr["loop"])
                cb = cpu_baseline_sdr_channel(sdr["ch_corr"])
                if cb:
                    out["sdr_channel"]["cpu_baseline"] = cb
        write_detail(out)
        print(json.dumps(result_line(out), separators=(",", ":")), flush=True)
    dist.close()


if __name__ == "__main__":
    main()
