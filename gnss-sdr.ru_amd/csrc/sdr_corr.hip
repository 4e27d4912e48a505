// sdr_corr.hip -- GPS-SDR tracking correlator (Correlator class) on gfx950.
//
// Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/objects/correlator.cpp
//   Accum        :425-448  wipe-off (sse_cmulsc, >>14) then sse_prn_accum_new: int32 E/P/L
//   Correlate    :160-237  per 2048-sample packet: accumulate to the code rollover,
//                          dump, continue (at most two dumps per packet)
//   UpdateState  :369-422  fp64 code / carrier phase, epoch counters, uint32 rollover
//   DumpAccum    :452-525  fp64 rotation by the wipe-off frequency error, floor to int32,
//                          Channel::Accum feedback, next code / carrier bins
//   SamplePRN    :562-590  101 fractional-chip code rows per SV (fp32 phase)
//   constructor  :63-98    3001 carrier rows, sine_gen at -IF - 10 Hz*k (fp32 phase)
//
// GPU part: sdr_accum_kernel runs a batch of Accum jobs (any channels, any
// receivers) -- one workgroup per job, samples strided over the threads, the
// int32 sums reduced with wavefront shuffles (integer addition is exact in any
// order).  Tables live in HBM: the carrier rows as packed CPX (49 MB), the
// code rows as a bit array (1.65 MB).  Host part: the Correlate schedule in
// phases, so each phase's Accum jobs of every channel go out as ONE launch;
// UpdateState / DumpAccum (fp64 scalar work + the channel callback) stay on the
// host exactly as restated from the reference.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "gnsscorr_internal.h"
#include "sdr_corr_state.h"

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      gnsscorr_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                     \
      return GNSSCORR_EDEVICE;                                                          \
    }                                                                                   \
  } while (0)

namespace {

using namespace sdrc;

// One Accum job per workgroup.  The same computation as sdrc::accum_block (the
// device-resident loop's segment, sdr_channel.hip), written out here: through
// the shared function the compiler schedules more loads in flight for this
// kernel (73 instead of 50 VGPRs, 6 instead of 8 waves per SIMD), and 4096 jobs
// take 17.5 instead of 15.2 us (same-box A/B).  test_sdr_track_gpu.py checks the
// two bit for bit (the loop against the host schedule, which launches this).
__global__ __launch_bounds__(kThreads) void sdr_accum_kernel(
    const uint32_t* __restrict__ packets, const gnsscorr_sdr_accum_job* __restrict__ jobs,
    const uint32_t* __restrict__ carrier, const uint32_t* __restrict__ codebits, int saturate,
    gnsscorr_sdr_corr* __restrict__ out) {
  __shared__ int32_t red[kThreads / 64][6];
  const gnsscorr_sdr_accum_job j = jobs[blockIdx.x];
  const uint32_t* d = packets + (size_t)j.packet * kN + j.data_off;
  const uint32_t* sn = carrier + (size_t)j.sbin * kRow + j.soff;
  size_t cb[3];
#pragma unroll
  for (int k = 0; k < 3; k++) cb[k] = ((size_t)j.sv * kCBins + j.cbin[k]) * kRow + j.coff[k];
  uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
  // Wave w covers the contiguous samples [1024 w, 1024 w + 1024) of the job,
  // 64 per step.  The code bits it needs per arm lie in the 33 words from
  // (cb + 1024 w) >> 5: lane l holds word l of that range (one coalesced load
  // per arm for the whole job), and each sample's bit comes from its word's
  // lane by ds_bpermute.
  static_assert(kThreads == 128 && kN == 2048, "two waves of 1024 samples");
  const int lane = threadIdx.x & 63, wave0 = (threadIdx.x >> 6) * 1024;
  const int nend = min(j.samps, wave0 + 1024);
  uint32_t cw[3];
  uint32_t sh[3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const size_t bit0 = cb[k] + (size_t)wave0;
    sh[k] = (uint32_t)bit0 & 31u;
    // words 0..32 cover bits up to sh + 1023; a lane loads only a word the
    // wave's samples reach (an idle wave loads nothing)
    const int last = ((int)sh[k] + (nend - wave0) - 1) >> 5;
    cw[k] = (wave0 < nend && lane <= last) ? codebits[(bit0 >> 5) + lane] : 0u;
  }
  // all 16 steps' packet and carrier words are loaded before the first is
  // used (a plain loop waited on memory latency at every step: one load pair
  // in flight per wave)
  constexpr int kSteps = 1024 / 64;
  uint32_t av[kSteps], bv[kSteps];
#pragma unroll
  for (int st = 0; st < kSteps; st++) {
    const int n = wave0 + st * 64 + lane;
    av[st] = n < nend ? d[n] : 0u;
    bv[st] = n < nend ? sn[n] : 0u;
  }
#pragma unroll
  for (int st = 0; st < kSteps; st++) {
    const int n = wave0 + st * 64 + lane;
    const bool live = n < nend;
    const uint32_t a = av[st], b = bv[st];
    const int32_t ai = lo16(a), aq = hi16(a), bi = lo16(b), bq = hi16(b);
    const int32_t ti = (ai * bi - aq * bq + 8192) >> 14, tq = (ai * bq + aq * bi + 8192) >> 14;
    int32_t wi = saturate ? sat16(ti) : (int32_t)(int16_t)ti;
    int32_t wq = saturate ? sat16(tq) : (int32_t)(int16_t)tq;
    if (!live) wi = wq = 0;
    const uint32_t rel = (uint32_t)(st * 64 + lane);   // n - wave0 < 1024
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const uint32_t r = rel + sh[k];
      const uint32_t word = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((r >> 5) << 2), (int)cw[k]);
      const int32_t m = (int32_t)((word >> (r & 31u)) & 1u) - 1;   // 0: +code, -1: -code
      acc[2 * k] += (uint32_t)((wi ^ m) - m);       // A.i * code  (+-1)
      acc[2 * k + 1] += (uint32_t)((wq ^ m) - m);   // A.q * code
    }
  }
#pragma unroll
  for (int k = 0; k < 6; k++)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc[k] += (uint32_t)__shfl_xor((int)acc[k], o, 64);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 6; k++) red[threadIdx.x >> 6][k] = (int32_t)acc[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    gnsscorr_sdr_corr r;
    for (int k = 0; k < 3; k++) {
      uint32_t si = 0, sq = 0;
      for (int w = 0; w < kThreads / 64; w++) {
        si += (uint32_t)red[w][2 * k];
        sq += (uint32_t)red[w][2 * k + 1];
      }
      r.i[k] = (int32_t)si;
      r.q[k] = (int32_t)sq;
    }
    out[blockIdx.x] = r;
  }
}

// DumpAccum, correlator.cpp:452-525, with the channel callback between the
// rotation and ProcessFeedback
void dump(gnsscorr_sdr_chan* s, gnsscorr_sdr_corr* c, int ch, gnsscorr_sdr_dump_fn cb,
          void* user) {
  rotate(s, c);
  gnsscorr_sdr_feedback f;
  memset(&f, 0, sizeof f);
  if (cb) cb(user, ch, s, c, &f);
  after_feedback(s, c, f);
}

}  // namespace

struct gnsscorr_sdr_corr_ctx {
  gnsscorr_sdr_corr_cfg cfg;
  hipStream_t stream = nullptr;
  uint32_t *d_carrier = nullptr, *d_codebits = nullptr, *d_packets = nullptr;
  gnsscorr_sdr_accum_job* d_jobs = nullptr;
  gnsscorr_sdr_corr* d_out = nullptr;
  size_t cap_packets = 0, cap_jobs = 0;
  gnsscorr_sdr_accum_job* h_jobs = nullptr;   // pinned staging
  gnsscorr_sdr_corr* h_out = nullptr;
};

extern "C" int gnsscorr_sdr_corr_destroy(gnsscorr_sdr_corr_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_carrier);
  (void)hipFree(c->d_codebits);
  (void)hipFree(c->d_packets);
  (void)hipFree(c->d_jobs);
  (void)hipFree(c->d_out);
  (void)hipHostFree(c->h_jobs);
  (void)hipHostFree(c->h_out);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_corr_create(gnsscorr_sdr_corr_ctx** out,
                                        const gnsscorr_sdr_corr_cfg* cfg) {
  if (!out || !cfg) return GNSSCORR_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gnsscorr_set_error("gnsscorr_sdr_corr_create: no HIP device");
    return GNSSCORR_ENODEV;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    gnsscorr_set_error("gnsscorr_sdr_corr_create: device %d out of range", cfg->device);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(cfg->device));
  auto* c = new gnsscorr_sdr_corr_ctx();
  c->cfg = *cfg;
  const size_t ncar = (size_t)kSBins * kRow;
  // + 33 words: a wave's 33-word window (sdr_accum_kernel) starting in the
  // last row stays inside the allocation even before its lane clamp
  const size_t nbits = (size_t)kSV * kCBins * kRow, nwords = nbits / 32 + 33;
  std::vector<uint32_t> car(ncar), bits(nwords, 0u);
  // carrier rows: sine_gen(row, -IF_FREQUENCY - (float)k*CARRIER_SPACING, fs, 4096)
  for (int k = -kCarrBins; k <= kCarrBins; k++) {
    const float f = (float)(-kIF) - (float)k * (float)kCarrSpacing;
    gnsscorr_sdr_sine_gen((int16_t*)&car[(size_t)(k + kCarrBins) * kRow], f, 2048000.0, kRow);
  }
  // code rows (SamplePRN): phase -0.5 + lcv/50 chips, fp32 steps of CODE_RATE/fs
  uint8_t chips[1023];
  for (int sv = 0; sv < kSV; sv++) {
    gnsscorr_sdr_code_gen(sv, chips);
    for (int lcv = 0; lcv < kCBins; lcv++) {
      float phase = (float)(-0.5 + (float)lcv / (float)kCodeBins);
      const float step = (float)(1.023e6 * kInvFs);
      const size_t base = ((size_t)sv * kCBins + lcv) * kRow;
      for (int k = 0; k < kRow; k++, phase += step) {
        const int idx = (int)floorf(phase + 1023) % 1023;
        if (chips[idx]) bits[(base + k) >> 5] |= 1u << ((base + k) & 31);
      }
    }
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->d_carrier, ncar * 4);
  if (e == hipSuccess) e = hipMalloc(&c->d_codebits, nwords * 4);
  if (e == hipSuccess) e = hipMemcpy(c->d_carrier, car.data(), ncar * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(c->d_codebits, bits.data(), nwords * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    gnsscorr_set_error("gnsscorr_sdr_corr_create: %s", hipGetErrorString(e));
    gnsscorr_sdr_corr_destroy(c);
    return GNSSCORR_EDEVICE;
  }
  *out = c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_init_chan(gnsscorr_sdr_chan* s, int sv, int acq_code_phase,
                                      int acq_doppler, double packets_since_acq) {
  if (!s || sv < 0 || sv >= kSV) {
    gnsscorr_set_error("gnsscorr_sdr_init_chan: sv %d out of range 0..31", sv);
    return GNSSCORR_EINVAL;
  }
  // InitCorrelator, correlator.cpp:610-676 (carrier_phase_prev, never set there, is 0)
  memset(s, 0, sizeof *s);
  double dt = packets_since_acq;
  dt *= (double).001;
  dt *= (double)acq_doppler * (double)1.023e6 / (double)1.57542e9;
  double cp = (double)acq_code_phase * 1023.0 / 2048.0;
  cp += (double)1023 - dt + 2.5;
  cp = fmod(cp, (double)1023);
  s->sv = (uint32_t)sv;
  s->active = 1;
  s->code_phase = s->code_phase_mod = cp;
  s->code_nco = 1.023e6 + acq_doppler * 1.023e6 / 1.57542e9;
  s->carrier_nco = kIF + acq_doppler;
  s->rollover = (uint32_t)(int32_t)ceil(((double)1023 - cp) * 2048000.0 / s->code_nco);
  s->cbin[0] = code_bin(cp + 0.5);
  s->cbin[1] = code_bin(cp + 0.0);
  s->cbin[2] = code_bin(cp - 0.5);
  for (int k = 0; k < 3; k++) s->coff[k] = acq_code_phase;   // pcode[k] += inc
  s->sbin = carrier_bin(s->carrier_nco);
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_accum_dev(gnsscorr_sdr_corr_ctx* c, const int16_t* d_packets,
                                      int n_jobs, const gnsscorr_sdr_accum_job* d_jobs,
                                      gnsscorr_sdr_corr* d_out) {
  if (!c || !d_packets || !d_jobs || !d_out || n_jobs < 0) return GNSSCORR_EINVAL;
  if (n_jobs == 0) return GNSSCORR_OK;
  HIP_TRY(hipSetDevice(c->cfg.device));
  hipLaunchKernelGGL(sdr_accum_kernel, dim3(n_jobs), dim3(kThreads), 0, c->stream,
                     (const uint32_t*)d_packets, d_jobs, c->d_carrier, c->d_codebits,
                     c->cfg.saturate, d_out);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

static int ensure_jobs(gnsscorr_sdr_corr_ctx* c, size_t n) {
  if (n <= c->cap_jobs) return GNSSCORR_OK;
  (void)hipFree(c->d_jobs);
  (void)hipFree(c->d_out);
  (void)hipHostFree(c->h_jobs);
  (void)hipHostFree(c->h_out);
  c->d_jobs = nullptr; c->d_out = nullptr; c->h_jobs = nullptr; c->h_out = nullptr;
  c->cap_jobs = 0;
  HIP_TRY(hipMalloc(&c->d_jobs, n * sizeof(gnsscorr_sdr_accum_job)));
  HIP_TRY(hipMalloc(&c->d_out, n * sizeof(gnsscorr_sdr_corr)));
  HIP_TRY(hipHostMalloc(&c->h_jobs, n * sizeof(gnsscorr_sdr_accum_job), hipHostMallocDefault));
  HIP_TRY(hipHostMalloc(&c->h_out, n * sizeof(gnsscorr_sdr_corr), hipHostMallocDefault));
  c->cap_jobs = n;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_correlate(gnsscorr_sdr_corr_ctx* c, const int16_t* h_packets,
                                      int n_packets, int n_ch, const int32_t* h_rx,
                                      gnsscorr_sdr_chan* st, gnsscorr_sdr_corr* corr,
                                      gnsscorr_sdr_dump_fn cb, void* user) {
  if (!c || !h_packets || !st || !corr || n_packets < 1 || n_ch < 0) return GNSSCORR_EINVAL;
  if (n_ch == 0) return GNSSCORR_OK;
  HIP_TRY(hipSetDevice(c->cfg.device));
  int rc;
  if ((size_t)n_packets > c->cap_packets) {
    (void)hipFree(c->d_packets);
    c->d_packets = nullptr;
    c->cap_packets = 0;
    HIP_TRY(hipMalloc(&c->d_packets, (size_t)n_packets * kN * 4));
    c->cap_packets = (size_t)n_packets;
  }
  if ((rc = ensure_jobs(c, (size_t)n_ch))) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_packets, h_packets, (size_t)n_packets * kN * 4,
                         hipMemcpyHostToDevice, c->stream));
  // per-channel progress through the packet (Correlate, correlator.cpp:183-235)
  std::vector<int32_t> off(n_ch, 0), left(n_ch, kN), dumps(n_ch, 0), job_of(n_ch, -1);
  std::vector<char> live(n_ch), dump_after(n_ch, 0);
  for (int ch = 0; ch < n_ch; ch++) {
    live[ch] = st[ch].active != 0;
    const int rx = h_rx ? h_rx[ch] : 0;
    if (live[ch] && (rx < 0 || rx >= n_packets)) {
      gnsscorr_set_error("gnsscorr_sdr_correlate: channel %d reads packet %d of %d", ch, rx,
                         n_packets);
      return GNSSCORR_EINVAL;
    }
  }
  for (int phase = 0; phase < 3; phase++) {
    int nj = 0;
    for (int ch = 0; ch < n_ch; ch++) {
      if (!live[ch]) continue;
      gnsscorr_sdr_chan* s = &st[ch];
      int32_t samps;
      if (dumps[ch] < 2 && s->rollover <= (uint32_t)left[ch]) {
        samps = (int32_t)s->rollover;
        dump_after[ch] = 1;
      } else {
        samps = left[ch];
        dump_after[ch] = 0;
      }
      job_of[ch] = -1;
      if (samps > 0) {
        gnsscorr_sdr_accum_job& j = c->h_jobs[nj];
        j = make_job(*s, h_rx ? h_rx[ch] : 0, off[ch], samps);
        if (!job_in_range(j, n_packets)) {
          gnsscorr_set_error("gnsscorr_sdr_correlate: channel %d state out of the tables "
                             "(sv %d sbin %d soff %d)", ch, j.sv, j.sbin, j.soff);
          return GNSSCORR_EINVAL;
        }
        job_of[ch] = nj++;
      }
      off[ch] += samps;
      left[ch] -= samps;
    }
    if (nj > 0) {
      HIP_TRY(hipMemcpyAsync(c->d_jobs, c->h_jobs, nj * sizeof(gnsscorr_sdr_accum_job),
                             hipMemcpyHostToDevice, c->stream));
      if ((rc = gnsscorr_sdr_accum_dev(c, (const int16_t*)c->d_packets, nj, c->d_jobs, c->d_out)))
        return rc;
      HIP_TRY(hipMemcpyAsync(c->h_out, c->d_out, nj * sizeof(gnsscorr_sdr_corr),
                             hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
    }
    bool more = false;
    for (int ch = 0; ch < n_ch; ch++) {
      if (!live[ch]) continue;
      gnsscorr_sdr_chan* s = &st[ch];
      if (job_of[ch] >= 0) {
        const gnsscorr_sdr_corr& r = c->h_out[job_of[ch]];
        for (int k = 0; k < 3; k++) {
          corr[ch].i[k] = (int32_t)((uint32_t)corr[ch].i[k] + (uint32_t)r.i[k]);
          corr[ch].q[k] = (int32_t)((uint32_t)corr[ch].q[k] + (uint32_t)r.q[k]);
        }
        update_state(s, c->h_jobs[job_of[ch]].samps);
      }
      if (dump_after[ch]) {
        dump(s, &corr[ch], ch, cb, user);
        dumps[ch]++;
        if (!s->active) live[ch] = 0;
      } else {
        live[ch] = 0;   // packet finished for this channel
      }
      if (live[ch]) more = true;
    }
    if (!more) break;
  }
  return GNSSCORR_OK;
}

extern "C" void gnsscorr_sdr_corr_tables(const gnsscorr_sdr_corr_ctx* c, const uint32_t** carrier,
                                         const uint32_t** codebits, int* saturate) {
  *carrier = c->d_carrier;
  *codebits = c->d_codebits;
  *saturate = c->cfg.saturate;
}

extern "C" int gnsscorr_sdr_corr_sync(gnsscorr_sdr_corr_ctx* c) {
  if (!c) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" void* gnsscorr_sdr_corr_stream(gnsscorr_sdr_corr_ctx* c) {
  return c ? (void*)c->stream : nullptr;
}

extern "C" int gnsscorr_sdr_corr_device(const gnsscorr_sdr_corr_ctx* c) {
  return c ? c->cfg.device : -1;
}
