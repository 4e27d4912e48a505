// sdr_corr_state.h -- the GPS-SDR Correlator's bookkeeping and its Accum, shared
// by the host-scheduled path (sdr_corr.hip) and the device-resident loop
// (sdr_channel.hip, gnsscorr_sdr_track_dev).
//
// Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/objects/correlator.cpp
//   Correlate    :160-237  per 2048-sample packet: accumulate to the code rollover,
//                          dump, continue (at most two dumps per packet)
//   UpdateState  :369-422  fp64 code / carrier phase, epoch counters, uint32 rollover
//   Accum        :425-448  wipe-off (sse_cmulsc, >>14) then sse_prn_accum_new
//   DumpAccum    :452-525  fp64 rotation, Channel::Accum, ProcessFeedback, rebin
//   ProcessFeedback :530-555
// The bookkeeping is __host__ __device__ with FMA contraction off, so the host
// schedule and the device loop evaluate the same fp64 expressions as the
// reference's x86 build (cos / sin of the rotation come from the host libm
// resp. ocml: a last-bit difference reaches an output only if a rotated
// correlation lies within ~1e-11 of an integer).
#ifndef GNSSCORR_SDR_CORR_STATE_H
#define GNSSCORR_SDR_CORR_STATE_H
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>
#include "gnsscorr_internal.h"

namespace sdrc {

constexpr int kN = 2048;                 // SAMPS_MS
constexpr int kRow = 2 * kN;             // pre-sampled row length
constexpr int kIF = 38400;               // IF_FREQUENCY (signaldef.h:34)
constexpr int kCarrSpacing = 10;         // CARRIER_SPACING (config.h:82)
constexpr int kCarrBins = 1500;          // CARRIER_BINS = 15000 / 10
constexpr int kSBins = 2 * kCarrBins + 1;
constexpr int kCodeBins = 50;            // CODE_BINS (config.h:81)
constexpr int kCBins = 2 * kCodeBins + 1;
constexpr int kSV = 32;                  // MAX_SV
constexpr int kThreads = 128;            // one Accum job per 128-thread workgroup
constexpr double kInvFs = 4.882812500000000e-7;   // INVERSE_SAMPLE_FREQUENCY

__host__ __device__ __forceinline__ int16_t lo16(uint32_t v) { return (int16_t)(v & 0xFFFFu); }
__host__ __device__ __forceinline__ int16_t hi16(uint32_t v) { return (int16_t)(v >> 16); }
__host__ __device__ __forceinline__ int32_t sat16(int32_t v) {
  return v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
}

__host__ __device__ inline uint32_t code_bin(double phase) {
#pragma clang fp contract(off)
  int32_t b = (int32_t)floor(phase * kCodeBins + 0.5) + kCodeBins / 2;
  if (b < 0) b = 0;
  if (b > 2 * kCodeBins) b = 2 * kCodeBins;
  return (uint32_t)b;
}

__host__ __device__ inline uint32_t carrier_bin(double nco) {
#pragma clang fp contract(off)
  int32_t b = (int32_t)floor((nco - kIF) / kCarrSpacing + 0.5) + kCarrBins;
  if (b < 0) b = 0;
  if (b > 2 * kCarrBins) b = 2 * kCarrBins;
  return (uint32_t)b;
}

// fmod(x, 1.0) and fmod(x, 1023) without the library's iterative reduction
// (the device libm's fmod is a long loop): x - trunc(x) is exact for every
// finite x (the integer bits are removed from x's own significand), and for
// 0 <= x < 4 * 1023, x - 1023 n with n = trunc(x / 1023) fixed up by one step
// is exact by Sterbenz's lemma (1023 n <= x < 2 * 1023 n for n >= 1), so both
// equal fmod bit for bit (a zero result takes the sign of x, as fmod's); other
// x take fmod itself.
__host__ __device__ __forceinline__ double fmod_1(double x) {
#pragma clang fp contract(off)
  if (!isfinite(x)) return fmod(x, 1.0);
  const double r = x - trunc(x);
  return r == 0.0 ? copysign(0.0, x) : r;   // fmod's zero has the sign of x
}
__host__ __device__ __forceinline__ double fmod_1023(double x) {
#pragma clang fp contract(off)
  if (!(x >= 0.0 && x < 4.0 * 1023.0)) return fmod(x, 1023);
  double r = x - 1023.0 * trunc(x / 1023.0);
  if (r < 0.0) r += 1023.0;
  else if (r >= 1023.0) r -= 1023.0;
  return r;
}

__host__ __device__ inline void update_state(gnsscorr_sdr_chan* s, int32_t samps) {   // :369-422
#pragma clang fp contract(off)
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
  s->carrier_phase_mod = fmod_1(s->carrier_phase_mod);
  s->code_phase_mod = fmod_1023(s->code_phase_mod);
  s->rollover -= (uint32_t)samps;
  s->soff += samps;
  for (int k = 0; k < 3; k++) s->coff[k] += samps;
  s->scount += (uint32_t)samps;
}

__host__ __device__ inline void rebin(gnsscorr_sdr_chan* s) {   // tail of DumpAccum, :497-524
#pragma clang fp contract(off)
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

// DumpAccum's rotation of the correlations by the wipe-off frequency error (:455-482)
__host__ __device__ inline void rotate(gnsscorr_sdr_chan* s, gnsscorr_sdr_corr* c) {
#pragma clang fp contract(off)
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
}

// ProcessFeedback (:530-555) and the rest of DumpAccum after Channel::Accum (:488-525)
__host__ __device__ inline void after_feedback(gnsscorr_sdr_chan* s, gnsscorr_sdr_corr* c,
                                               const gnsscorr_sdr_feedback& f) {
  s->carrier_nco = f.carrier_nco;
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

// the Accum job of a correlator state: samps samples from data_off of packet
__host__ __device__ inline gnsscorr_sdr_accum_job make_job(const gnsscorr_sdr_chan& s, int packet,
                                                           int data_off, int samps) {
  gnsscorr_sdr_accum_job j;
  j.packet = packet;
  j.data_off = data_off;
  j.samps = samps;
  j.sv = (int32_t)s.sv;
  j.sbin = (int32_t)s.sbin;
  j.soff = s.soff;
  for (int k = 0; k < 3; k++) { j.cbin[k] = (int32_t)s.cbin[k]; j.coff[k] = s.coff[k]; }
  return j;
}

// the reference reads the pre-sampled rows through raw pointers: allow running
// into the next row, but not past the whole table
__host__ __device__ inline bool job_in_range(const gnsscorr_sdr_accum_job& j, int n_packets) {
  if (j.samps < 0 || j.samps > kN || j.data_off < 0 || j.data_off + j.samps > kN ||
      j.packet < 0 || j.packet >= n_packets || j.sv < 0 || j.sv >= kSV || j.sbin < 0 ||
      j.sbin >= kSBins)
    return false;
  const long long send = (long long)j.sbin * kRow + j.soff + j.samps;
  if (j.soff < 0 || send > (long long)kSBins * kRow) return false;
  for (int k = 0; k < 3; k++) {
    if (j.cbin[k] < 0 || j.cbin[k] >= kCBins || j.coff[k] < 0) return false;
    const long long cend = ((long long)j.sv * kCBins + j.cbin[k]) * kRow + j.coff[k] + j.samps;
    if (cend > (long long)kSV * kCBins * kRow) return false;
  }
  return true;
}

// Correlator::Accum of one job by ONE wavefront (sse_cmulsc >> 14 of the packet
// by the carrier row, then the E/P/L code bits; int32 wrapping sums), for the
// device-resident loop.  d: the job's packet (2048 CPX).  Every lane returns the
// six sums (xor-shuffle reduction, no LDS, no barrier).  The job is done as two
// halves of 1024 samples, 64 per step, exactly as a wave of sdr_accum_kernel
// does its half: per arm the code bits of a half lie in the 33 words from
// (cb + 1024 h) >> 5; lane l holds word l of that range (one coalesced load per
// arm) and each sample's bit comes from its word's lane by ds_bpermute.  All 16
// steps' packet and carrier words of a half are loaded before the first is used.
__device__ __forceinline__ gnsscorr_sdr_corr accum_wave(const gnsscorr_sdr_accum_job& j,
                                                       const uint32_t* __restrict__ d,
                                                       const uint32_t* __restrict__ carrier,
                                                       const uint32_t* __restrict__ codebits,
                                                       int saturate) {
  static_assert(kN == 2048, "two halves of 1024 samples");
  d += j.data_off;
  const uint32_t* sn = carrier + (size_t)j.sbin * kRow + j.soff;
  size_t cb[3];
#pragma unroll
  for (int k = 0; k < 3; k++) cb[k] = ((size_t)j.sv * kCBins + j.cbin[k]) * kRow + j.coff[k];
  uint32_t acc[6] = {0, 0, 0, 0, 0, 0};
  const int lane = threadIdx.x & 63;
  for (int h = 0; h < 2; h++) {
    const int wave0 = h * 1024;
    if (wave0 >= j.samps) break;   // wave-uniform
    const int nend = min(j.samps, wave0 + 1024);
    uint32_t cw[3];
    uint32_t sh[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const size_t bit0 = cb[k] + (size_t)wave0;
      sh[k] = (uint32_t)bit0 & 31u;
      const int last = ((int)sh[k] + (nend - wave0) - 1) >> 5;
      cw[k] = lane <= last ? codebits[(bit0 >> 5) + lane] : 0u;
    }
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
  }
#pragma unroll
  for (int k = 0; k < 6; k++)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc[k] += (uint32_t)__shfl_xor((int)acc[k], o, 64);
  gnsscorr_sdr_corr r;
  for (int k = 0; k < 3; k++) {
    r.i[k] = (int32_t)acc[2 * k];
    r.q[k] = (int32_t)acc[2 * k + 1];
  }
  return r;
}

}  // namespace sdrc

extern "C" {
/* the context's resident tables (sdr_corr.hip), for the device loop */
void gnsscorr_sdr_corr_tables(const gnsscorr_sdr_corr_ctx* c, const uint32_t** carrier,
                              const uint32_t** codebits, int* saturate);
}
#endif
