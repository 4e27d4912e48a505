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

constexpr int kN = 2048;                 // SAMPS_MS
constexpr int kRow = 2 * kN;             // pre-sampled row length
constexpr int kIF = 38400;               // IF_FREQUENCY (signaldef.h:34)
constexpr int kCarrSpacing = 10;         // CARRIER_SPACING (config.h:82)
constexpr int kCarrBins = 1500;          // CARRIER_BINS = 15000 / 10
constexpr int kSBins = 2 * kCarrBins + 1;
constexpr int kCodeBins = 50;            // CODE_BINS (config.h:81)
constexpr int kCBins = 2 * kCodeBins + 1;
constexpr int kSV = 32;                  // MAX_SV
constexpr int kThreads = 128;
constexpr double kInvFs = 4.882812500000000e-7;   // INVERSE_SAMPLE_FREQUENCY

__device__ __forceinline__ int16_t lo16(uint32_t v) { return (int16_t)(v & 0xFFFFu); }
__device__ __forceinline__ int16_t hi16(uint32_t v) { return (int16_t)(v >> 16); }
__device__ __forceinline__ int32_t sat16(int32_t v) {
  return v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
}

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

// ---- host restatement of the Correlator bookkeeping -------------------------
uint32_t code_bin(double phase) {
  int32_t b = (int32_t)floor(phase * kCodeBins + 0.5) + kCodeBins / 2;
  if (b < 0) b = 0;
  if (b > 2 * kCodeBins) b = 2 * kCodeBins;
  return (uint32_t)b;
}

uint32_t carrier_bin(double nco) {
  int32_t b = (int32_t)floor((nco - kIF) / kCarrSpacing + 0.5) + kCarrBins;
  if (b < 0) b = 0;
  if (b > 2 * kCarrBins) b = 2 * kCarrBins;
  return (uint32_t)b;
}

void update_state(gnsscorr_sdr_chan* s, int32_t samps) {   // correlator.cpp:369-422
  s->code_phase += samps * s->code_nco * kInvFs;
  s->carrier_phase += samps * s->carrier_nco * kInvFs;
  s->code_phase_mod += samps * s->code_nco * kInvFs;
  s->carrier_phase_mod += samps * s->carrier_nco * kInvFs;
  const uint32_t inc = s->code_phase_mod >= 2.0 * 1023.0 ? 2u : (s->code_phase_mod >= 1023.0 ? 1u : 0u);
  if (inc) {
    s->epoch_1ms += inc;
    if (s->epoch_1ms >= 20) {
      s->epoch_1ms %= 20;
      if (++s->epoch_20ms >= 300) {
        s->epoch_20ms = 0;
        s->z_count += 6;
        if (s->z_count > 604800.0) s->z_count = 0;
      }
    }
  }
  s->carrier_phase_mod = fmod(s->carrier_phase_mod, 1.0);
  s->code_phase_mod = fmod(s->code_phase_mod, 1023);
  s->rollover -= (uint32_t)samps;
  s->soff += samps;
  for (int k = 0; k < 3; k++) s->coff[k] += samps;
  s->scount += (uint32_t)samps;
}

void rebin(gnsscorr_sdr_chan* s) {   // tail of DumpAccum, correlator.cpp:497-524
  const double r = ceil(((double)1023 - s->code_phase_mod) * 2048000.0 / s->code_nco);
  s->rollover = isfinite(r) ? (uint32_t)(int32_t)r : 0x80000000u;   // (int32)inf on x86
  s->cbin[0] = code_bin(s->code_phase_mod + 0.5);
  s->cbin[1] = code_bin(s->code_phase_mod + 0.0);
  s->cbin[2] = code_bin(s->code_phase_mod - 0.5);
  s->coff[0] = s->coff[1] = s->coff[2] = 0;
  s->sbin = carrier_bin(s->carrier_nco);
  s->soff = 0;
  s->scount = 0;
}

void dump(gnsscorr_sdr_chan* s, gnsscorr_sdr_corr* c, int ch, gnsscorr_sdr_dump_fn cb,
          void* user) {   // DumpAccum, correlator.cpp:452-496
  // f1 in uint32 arithmetic as the reference (sbin is uint32): wraps below the centre bin
  const double f1 = (double)((s->sbin - (uint32_t)kCarrBins) * (uint32_t)kCarrSpacing + (uint32_t)kIF);
  const double fix = 3.141592653589793 * (s->carrier_nco - f1) * (double)s->scount * kInvFs;
  double ang = s->carrier_phase_prev * 6.283185307179586 + fix;
  ang = -ang;
  const double ca = cos(ang), sa = sin(ang);
  s->carrier_phase_prev = s->carrier_phase_mod;
  for (int k = 0; k < 3; k++) {
    const double tI = c->i[k], tQ = c->q[k];
    c->i[k] = (int32_t)floor(ca * tI - sa * tQ);
    c->q[k] = (int32_t)floor(sa * tI + ca * tQ);
  }
  gnsscorr_sdr_feedback f;
  memset(&f, 0, sizeof f);
  if (cb) cb(user, ch, s, c, &f);
  s->carrier_nco = f.carrier_nco;   // ProcessFeedback, correlator.cpp:530-555
  s->code_nco = f.code_nco;
  s->navigate = f.navigate;
  if (f.reset_1ms) s->epoch_1ms = 0;
  if (f.reset_20ms) s->epoch_20ms = 60;
  if (f.set_z_count) s->z_count = f.z_count;
  if (f.kill) memset(s, 0, sizeof *s);
  s->count++;
  memset(c, 0, sizeof *c);
  rebin(s);
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

static bool job_in_range(const gnsscorr_sdr_accum_job& j, int n_packets) {
  if (j.samps < 0 || j.samps > kN || j.data_off < 0 || j.data_off + j.samps > kN ||
      j.packet < 0 || j.packet >= n_packets || j.sv < 0 || j.sv >= kSV || j.sbin < 0 ||
      j.sbin >= kSBins)
    return false;
  // the reference reads rows through raw pointers: allow running into the next
  // row, but not past the whole table
  const long long send = (long long)j.sbin * kRow + j.soff + j.samps;
  if (j.soff < 0 || send > (long long)kSBins * kRow) return false;
  for (int k = 0; k < 3; k++) {
    if (j.cbin[k] < 0 || j.cbin[k] >= kCBins || j.coff[k] < 0) return false;
    const long long cend = ((long long)j.sv * kCBins + j.cbin[k]) * kRow + j.coff[k] + j.samps;
    if (cend > (long long)kSV * kCBins * kRow) return false;
  }
  return true;
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
        j.packet = h_rx ? h_rx[ch] : 0;
        j.data_off = off[ch];
        j.samps = samps;
        j.sv = (int32_t)s->sv;
        j.sbin = (int32_t)s->sbin;
        j.soff = s->soff;
        for (int k = 0; k < 3; k++) { j.cbin[k] = (int32_t)s->cbin[k]; j.coff[k] = s->coff[k]; }
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
