// sdr_channel.hip -- the GPS-SDR Channel object (bit lock, frame sync, parity,
// C/N0 and the channel's FLL/PLL/DLL) batched over channels on gfx950
// (SURVEY 8(f) ranks 2 and 4).
//
// Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/objects/
//   channel.cpp  Clear :71-130, Start :133-170, Accum :182-279,
//                DumpAccum :282-318, EstCN0 :322-355, FrequencyLock :359-417,
//                DLL :422-447, PLL :452-497, Epoch :502-518, BitLock :524-611,
//                BitStuff :615-651, ProcessDataBit :655-727, FrameSync :731-780,
//                ParityCheck :784-812, ValidFrameFormat :818-904, PLL_W :909-927,
//                DLL_W :931-941, Error :945-985, Kill :988-993
//   fft.cpp      FFT(512) with every rank scaled, initW :121-149, doFFT :182-205
//   x86.cpp      x86_cmag :255-269
//
// One thread per channel runs its 1-ms calls in order (the object is a serial
// state machine); channels are independent.  The channel logic is written once
// as __host__ __device__ code: gnsscorr_sdr_channel_start runs the same Clear /
// Start on the host.  Float and double follow the reference's expression types
// (e.g. carrier_nco = IF_FREQUENCY + aPLL.z is a float sum), FMA contraction off.
// Two reads of indeterminate values in the reference are given fixed values:
// PLL's `cross` (an uninitialised local; it feeds only aPLL.fll_lock, which no
// output reads) is 0, and EstCN0's NP when WBP == 0 (all-zero buffers) is 0.
#include <hip/hip_runtime.h>
#include <math.h>
#include <string.h>
#include <stdlib.h>
#include "gnsscorr_internal.h"
#include "sdr_corr_state.h"

#pragma clang fp contract(off)

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

constexpr int kEmpty = 0, kNormal = 3;          // Channel_State (channel.h:33-39)
constexpr int kFreqLockPoints = 512;            // FREQ_LOCK_POINTS (channel.h:41)
constexpr uint32_t kPreamble = 0x8B;            // PREAMBLE (defines.h:117)
constexpr double kCodeRate = 1.023e6;           // CODE_RATE (defines.h:147)
constexpr double kL1 = 1.57542e9;               // L1 (defines.h:137)
constexpr double kInvL1 = 6.347513678891978e-10;  // INVERSE_L1 (defines.h:145)
constexpr double kTwoPi = 6.283185307179586;    // TWO_PI (defines.h:104)
constexpr int kIF = 38400;                      // IF_FREQUENCY (signaldef.h:34)
constexpr int kCarrierLimit = 1500 * 10;        // CARRIER_BINS * CARRIER_SPACING (config.h:82-83)
enum { PLLBW, FLLBW, A3, B3, W0P, W0P2, W0P3, A2, W0F, W0F2, GAIN, PW, PX, PZ, PLL_LOCK, FLL_LOCK, PT };
enum { DLLBW, DX, DZ, DA, DW0, DW02, DT };

struct Twiddles { uint32_t w[kFreqLockPoints / 2]; };   // FFT(512) forward W: (c, s) int16

typedef gnsscorr_sdr_channel Chan;

__host__ __device__ inline uint32_t rotl(uint32_t x, int n) { return (x << n) ^ (x >> (32 - n)); }

__host__ __device__ inline void pll_w(Chan& s, float bw) {   // channel.cpp:909-927
  float* p = s.pll;
  p[PLLBW] = bw;
  p[FLLBW] = 4.0f;
  p[B3] = 2.40f;
  p[A3] = 1.10f;
  p[A2] = 1.414f;
  p[W0P] = (float)(p[PLLBW] / 0.7845);
  p[W0P2] = p[W0P] * p[W0P];
  p[W0P3] = p[W0P2] * p[W0P];
  p[W0F] = (float)(p[FLLBW] / 0.53);
  p[W0F2] = p[W0F] * p[W0F];
  p[GAIN] = 1.0f;
  p[PT] = (float)(.001 * (float)s.len);
}

__host__ __device__ inline void dll_w(Chan& s, float bw) {   // channel.cpp:931-941
  float* d = s.dll;
  d[DLLBW] = bw;
  d[DA] = 1.414f;
  d[DW0] = (float)(d[DLLBW] / 0.7845);
  d[DW02] = d[DW0] * d[DW0];
  d[DT] = (float)(.001 * (float)s.len);
}

// Channel::Clear (channel.cpp:71-130).  Its memset of valid_frame writes
// 5*sizeof(int32) bytes over bool valid_frame[5] and runs on into navigate,
// z_lock, converged, frame_z, z_count and z_count_pend: z_count_pend is zeroed
// too.  chan, carrier_nco and code_nco are left as they are.
__host__ __device__ inline void clear(Chan& s, uint32_t* fft) {
  s.len = 1;
  s.count = 0;
  s.state = kEmpty;
  s.sv = 666;
  for (int k = 0; k < 17; k++) s.pll[k] = 0.0f;
  for (int k = 0; k < 7; k++) s.dll[k] = 0.0f;
  for (int k = 0; k < 3; k++) s.I[k] = s.Q[k] = s.P[k] = 1;
  s.I_prev = s.Q_prev = 1;
  s.I_avg = 1.0f;
  s.Q_var = 1.0f;
  s.P_avg = 8e4f;
  s.cn0 = 40.0f;
  s.bit_lock = s.bit_lock_pend = s.bit_lock_ticks = 0;
  s.I_sum20 = s.Q_sum20 = 0;
  for (int k = 0; k < 20; k++) s.I_buff[k] = s.Q_buff[k] = s.P_buff[k] = 0;
  s.epoch_20ms = s.epoch_1ms = s.best_epoch = 0;
  for (int k = 0; k < 5; k++) s.valid_frame[k] = 0;
  s.converged = s.navigate = s.z_lock = 0;
  s.frame_z = s.z_count = s.z_count_pend = 0;
  for (int k = 0; k < 12; k++) s.word_buff[k] = 0;
  s.frame_lock = s.frame_lock_pend = 0;
  s.bit_number = s.subframe = 0;
  s.freq_lock_ticks = 0;
  s.freq_lock = 0;
  for (int k = 0; k < kFreqLockPoints; k++) fft[k] = 0;
}

__host__ __device__ inline void kill(Chan& s, uint32_t* fft) {   // channel.cpp:988-993
  s.state = kEmpty;
  clear(s, fft);
}

// ---- integer FFT(512): every rank scaled (fft.cpp:55-81, 182-205, 403-441)
__device__ void fft512(uint32_t* x, const Twiddles& tw) {
  for (int k = 0; k < kFreqLockPoints; k++) {   // doShuffle
    const int j = (int)(__brev((uint32_t)k) >> 23);
    if (j > k) {
      const uint32_t t = x[k];
      x[k] = x[j];
      x[j] = t;
    }
  }
  int bsize = 1, nblocks = kFreqLockPoints >> 1;
  for (int r = 0; r < 9; r++) {
    for (int blk = 0; blk < nblocks; blk++)
      for (int j = 0; j < bsize; j++) {
        const int a = blk * 2 * bsize + j, b = a + bsize;
        const uint32_t w = tw.w[j * nblocks];
        const int32_t wi = (int16_t)(w & 0xFFFF), wq = (int16_t)(w >> 16);
        const uint32_t A = x[a], B = x[b];
        const int16_t ai = (int16_t)((int16_t)(A & 0xFFFF) >> 1), aq = (int16_t)((int16_t)(A >> 16) >> 1);
        const int16_t bi0 = (int16_t)((int16_t)(B & 0xFFFF) >> 1), bq0 = (int16_t)((int16_t)(B >> 16) >> 1);
        int32_t bi = (int32_t)bi0 * wi - (int32_t)bq0 * wq;
        int32_t bq = (int32_t)bi0 * wq + (int32_t)bq0 * wi;
        bi = (bi + 8192) >> 14;
        bq = (bq + 8192) >> 14;
        x[b] = (uint32_t)(uint16_t)(int16_t)(ai - (int16_t)bi) |
               (uint32_t)(uint16_t)(int16_t)(aq - (int16_t)bq) << 16;
        x[a] = (uint32_t)(uint16_t)(int16_t)(ai + (int16_t)bi) |
               (uint32_t)(uint16_t)(int16_t)(aq + (int16_t)bq) << 16;
      }
    bsize <<= 1;
    nblocks >>= 1;
  }
}

__device__ void frequency_lock(Chan& s, uint32_t* fft, const Twiddles& tw) {   // :359-417
  const int32_t it = s.I[1] >> 3, qt = s.Q[1] >> 3;
  if (s.count > 1000) {
    const uint32_t ui = (uint32_t)it, uq = (uint32_t)qt;   // int32 wrap
    const int16_t fi = (int16_t)(ui * ui - uq * uq), fq = (int16_t)(2u * ui * uq);
    fft[s.freq_lock_ticks] = (uint32_t)(uint16_t)fi | (uint32_t)(uint16_t)fq << 16;
    s.freq_lock_ticks++;
  }
  if (s.freq_lock_ticks >= kFreqLockPoints) {
    fft512(fft, tw);
    int32_t mx = 0, mind = 0;
    for (int k = 0; k < kFreqLockPoints; k++) {   // x86_cmag + peak (first strict max)
      const int32_t i = (int16_t)(fft[k] & 0xFFFF), q = (int16_t)(fft[k] >> 16);
      const int32_t p = (int32_t)((uint32_t)i * (uint32_t)i + (uint32_t)q * (uint32_t)q);
      fft[k] = (uint32_t)p;
      if (p > mx) { mx = p; mind = k; }
    }
    if (mind >= kFreqLockPoints / 2) mind -= kFreqLockPoints;
    float df = (float)(1000.0 / ((float)2.0 * s.len));
    df /= (float)kFreqLockPoints;
    df *= (float)mind;
    s.dll[DX] = (float)(s.dll[DX] + 2.0 * df * kCodeRate / kL1);
    s.pll[PX] = (float)(s.pll[PX] + 2.0 * df);
    s.freq_lock = 1;
    s.freq_lock_ticks = 0;
  }
}

__device__ void pll(Chan& s) {   // channel.cpp:452-497 (FLL terms: df = 0, cross = 0)
  float* p = s.pll;
  double dp = 0, df = 0;
  const double cross = 0.0;
  if (s.I[1] != 0) dp = atan((double)s.Q[1] / (double)s.I[1]) / kTwoPi;
  p[PLL_LOCK] = (float)(p[PLL_LOCK] + (dp - p[PLL_LOCK]) * .1);
  p[PLL_LOCK] = (float)dp;
  p[FLL_LOCK] = (float)(p[FLL_LOCK] + (cross / s.P_avg - p[FLL_LOCK]) * .1);
  p[PW] = (float)(p[PW] + p[PT] * (p[W0P3] * dp + p[W0F2] * df));
  p[PX] = (float)(p[PX] + p[PT] * (0.5 * p[PW] + (p[A2] * p[W0F]) * df + (p[A3] * p[W0P2]) * dp));
  p[PZ] = (float)(0.5 * p[PX] + (p[B3] * p[W0P]) * dp);
  s.carrier_nco = (double)((float)kIF + p[PZ]);
}

__device__ void dll(Chan& s) {   // channel.cpp:422-447
  const double ep = sqrt((double)s.P[0]), lp = sqrt((double)s.P[2]);
  const double sp = sqrt((double)(int32_t)((uint32_t)s.P[2] + (uint32_t)s.P[0]));
  const double code_err = (ep - lp) / sp;
  if ((s.count < 1000) && (s.P_avg < 8e4))
    s.code_nco = kCodeRate + (0.5 * s.pll[PX] * kCodeRate * kInvL1) - 5.0;
  else
    s.code_nco = kCodeRate + (0.5 * s.pll[PX] * kCodeRate * kInvL1) + code_err;
}

__device__ void error_check(Chan& s, uint32_t* fft) {   // channel.cpp:945-985
  if ((s.P_avg < 8e4) && (s.count > 1000)) kill(s, fft);
  if ((s.count == 15000) && !s.bit_lock && s.freq_lock) {
    s.freq_lock_ticks = 0;
    s.freq_lock = 0;
  }
  if ((s.count > 30000) && !s.converged) kill(s, fft);
  if (fabs(s.carrier_nco - kIF) > kCarrierLimit) kill(s, fft);
  if (s.bit_lock) {
    if ((s.cn0 > 39.0) && (s.len != 1)) {
      s.len = 1;
      pll_w(s, 18.0f);
    }
    if ((s.cn0 < 37.0) && (s.len != 20)) {
      s.len = 20;
      pll_w(s, 18.0f);
    }
  }
}

__device__ void dump_accum(Chan& s, uint32_t* fft, const Twiddles& tw) {   // :282-318
  for (int k = 0; k < 3; k++)
    s.P[k] = (int32_t)((uint32_t)s.I[k] * (uint32_t)s.I[k] + (uint32_t)s.Q[k] * (uint32_t)s.Q[k]);
  s.I_avg = (float)(s.I_avg + (fabsf((float)s.I[1]) - s.I_avg) * .02);
  s.Q_var = (float)(s.Q_var + ((float)s.Q[1] * (float)s.Q[1] - s.Q_var) * .02);
  s.P_avg = (float)(s.P_avg + ((float)s.P[1] / s.len - s.P_avg) * .02);
  if (!s.freq_lock) frequency_lock(s, fft, tw);
  else pll(s);
  dll(s);
  error_check(s, fft);
  s.I_prev = s.I[1];
  s.Q_prev = s.Q[1];
  s.I[0] = s.I[1] = s.I[2] = 0;
  s.Q[0] = s.Q[1] = s.Q[2] = 0;
}

__device__ void est_cn0(Chan& s) {   // channel.cpp:322-355
  if ((s.epoch_1ms == 19) && s.bit_lock) {
    const float nbp = (float)(int32_t)((uint32_t)s.I_sum20 * (uint32_t)s.I_sum20 +
                                       (uint32_t)s.Q_sum20 * (uint32_t)s.Q_sum20);
    float wbp = 0.0f;
    for (int k = 0; k < 20; k++)
      wbp += (float)(int32_t)((uint32_t)s.I_buff[k] * (uint32_t)s.I_buff[k] +
                              (uint32_t)s.Q_buff[k] * (uint32_t)s.Q_buff[k]);
    float np = 0.0f;
    if (wbp > 0.0) np = nbp / wbp;
    if ((np - 1.0) / (20.0 - np) > 0.0) {
      const float ncn0 = (float)(10 * log10((np - 1.0) / (20.0 - np)) + 30.0 + .25);
      s.cn0 = (float)(s.cn0 + (ncn0 - s.cn0) * .02);
    }
    if (s.cn0 < 15.0) s.cn0 = 15.0f;
  }
}

__device__ void bit_lock(Chan& s) {   // channel.cpp:524-611
  const int32_t thresh_high = 100, thresh_low = 25;
  if (s.epoch_1ms == 19) {
    if (!s.bit_lock) {
      int32_t err = 0, new_epoch = 0;
      for (int k = 0; k < 20; k++) {
        if (s.P_buff[k] > thresh_high) {
          s.bit_lock = 1;
          new_epoch = k;
        }
        if (s.P_buff[k] > thresh_low) err++;
      }
      if (s.bit_lock) {
        s.best_epoch = 19;
        s.bit_lock_pend = 1;
        s.bit_lock_ticks = 0;
        s.epoch_1ms = (38 - new_epoch) % 20;
        int32_t pb[20];
        for (int k = 0; k < 20; k++) pb[k] = s.P_buff[k];
        for (int k = 0; k < 20; k++) s.P_buff[k] = pb[(k + new_epoch + 1) % 20];
      }
      if (err > 1) {
        s.best_epoch = 0;
        s.bit_lock_ticks = 0;
        s.bit_lock = 0;
        s.frame_lock = 0;
        for (int k = 0; k < 20; k++) s.P_buff[k] = 0;
      }
    } else if (s.bit_lock_ticks < 60000) {
      int32_t err = 0, new_epoch = 0;
      for (int k = 0; k < 20; k++)
        if (s.P_buff[k] > err) {
          err = s.P_buff[k];
          new_epoch = k;
        }
      if (new_epoch != 19) {
        s.best_epoch = 0;
        s.bit_lock_ticks = 0;
        s.bit_lock = 0;
        s.frame_lock = 0;
        for (int k = 0; k < 20; k++) s.P_buff[k] = 0;
      }
    }
  }
  s.bit_lock_ticks++;
}

__host__ __device__ inline bool parity_check(uint32_t w) {   // channel.cpp:784-812
  const uint32_t d1 = w & 0xFBFFBF00u, d2 = rotl(w, 1) & 0x07FFBF01u;
  const uint32_t d3 = rotl(w, 2) & 0xFC0F8100u, d4 = rotl(w, 3) & 0xF81FFE02u;
  const uint32_t d5 = rotl(w, 4) & 0xFC00000Eu, d6 = rotl(w, 5) & 0x07F00001u;
  const uint32_t d7 = rotl(w, 6) & 0x00003000u;
  const uint32_t t = d1 ^ d2 ^ d3 ^ d4 ^ d5 ^ d6 ^ d7;
  const uint32_t par = (t ^ rotl(t, 6) ^ rotl(t, 12) ^ rotl(t, 18) ^ rotl(t, 24)) & 0x3Fu;
  return par == (w & 0x3Fu);
}

// preamble / sid / zero bits of a (TLM, HOW) pair, inverted per bit 30 (:738-768)
__device__ inline bool tlm_how_ok(uint32_t w0, uint32_t w1, uint32_t* sid_out) {
  uint32_t pre = (w0 >> 22) & 0xFFu, sid = (w1 >> 8) & 7u, zero = w1 & 3u;
  if (w0 & 0x40000000u) {
    pre ^= 0xFFu;
    zero ^= 3u;
  }
  if (w1 & 0x40000000u) sid ^= 7u;
  *sid_out = sid;
  return pre == kPreamble && sid >= 1 && sid <= 5 && zero == 0;
}

__device__ bool frame_sync(uint32_t w0, uint32_t w1) {   // channel.cpp:731-780
  uint32_t sid;
  if (!tlm_how_ok(w0, w1, &sid)) return false;
  if (w0 & 0x40000000u) w0 ^= 0x3FFFFFC0u;
  if (w1 & 0x40000000u) w1 ^= 0x3FFFFFC0u;
  return parity_check(w0) && parity_check(w1);
}

__device__ bool valid_frame_format(uint32_t* sf) {   // channel.cpp:818-904 (modifies sf)
  uint32_t sid, next_sid;
  if (!tlm_how_ok(sf[0], sf[1], &sid)) return false;
  if (!tlm_how_ok(sf[10], sf[11], &next_sid)) return false;
  if ((next_sid - sid) != 1u && (next_sid - sid) != (uint32_t)-4) return false;
  for (int k = 0; k < 12; k++)
    if (sf[k] & 0x40000000u) sf[k] ^= 0x3FFFFFC0u;
  int errs = 0;
  for (int k = 0; k < 12; k++)
    if (!parity_check(sf[k])) errs++;
  return errs == 0;
}

struct Events {
  gnsscorr_sdr_subframe* ev;
  int max;
  int32_t* n;
  int chan, ms;
};

__device__ void process_data_bit(Chan& s, const Events& e) {   // channel.cpp:655-727
  if (!s.frame_lock) {
    if (frame_sync(s.word_buff[10], s.word_buff[11])) {
      s.frame_lock = 1;
      s.frame_lock_pend = 1;
      s.bit_number = 299;
      s.epoch_20ms = 60;
    }
  }
  if (s.frame_lock) {
    s.bit_number = (s.bit_number + 1) % 300;
    if (s.bit_number == 0) {
      uint32_t sf[12];
      for (int k = 0; k < 12; k++) sf[k] = s.word_buff[k];
      bool reset = true;
      if (valid_frame_format(sf)) {
        const int32_t sid = (int32_t)((sf[1] >> 8) & 7u);
        s.frame_z = 4 * (int32_t)((sf[1] >> 13) & 0x1FFFFu);
        if (sid > 0 && sid < 6) {
          reset = false;
          s.subframe = sid;
          s.valid_frame[sid - 1] = 1;
          const int slot = atomicAdd(e.n, 1);   // the pipe write to the ephemeris task (:687)
          if (slot < e.max) {
            gnsscorr_sdr_subframe o;
            o.sv = s.sv;
            o.subframe = sid;
            for (int k = 0; k < 12; k++) o.word_buff[k] = sf[k];
            o.chan = e.chan;
            o.ms = e.ms;
            e.ev[slot] = o;
          }
          if (!s.z_lock) {
            s.z_count_pend = 1;
            s.z_count = 3 * s.frame_z / 2;
            s.z_lock = 1;
            s.navigate = 1;
            s.converged = 1;
          }
        }
      }
      if (reset) {
        s.subframe = 0;
        for (int k = 0; k < 5; k++) s.valid_frame[k] = 0;
        s.frame_lock = 0;
      }
    }
  }
}

__device__ void bit_stuff(Chan& s, const Events& e) {   // channel.cpp:615-651
  if (s.bit_lock && (s.epoch_1ms == 19)) {
    const uint32_t temp_bit = s.I_sum20 > 0 ? 1u : 0u;
    for (int k = 0; k <= 10; k++) s.word_buff[k] = (s.word_buff[k] << 1) + ((s.word_buff[k + 1] >> 29) & 1u);
    s.word_buff[11] = (s.word_buff[11] << 1) + temp_bit;
    process_data_bit(s, e);
  }
}

__device__ void epoch(Chan& s) {   // channel.cpp:502-518
  s.epoch_1ms++;
  if (s.epoch_1ms >= 20) {
    s.epoch_1ms = 0;
    s.epoch_20ms++;
    if (s.epoch_20ms >= 300) {
      s.z_count += 6;
      s.epoch_20ms = 0;
    }
  }
  s.count++;
}

// Channel::Accum (channel.cpp:182-279)
__device__ void accum(Chan& s, uint32_t* fft, const Twiddles& tw, gnsscorr_sdr_corr c,
                      gnsscorr_sdr_feedback* fb, const Events& e) {
  for (int k = 0; k < 3; k++) {
    c.i[k] >>= 2;
    c.q[k] >>= 2;
  }
  for (int k = 0; k < 3; k++) {
    s.I[k] = (int32_t)((uint32_t)s.I[k] + (uint32_t)c.i[k]);
    s.Q[k] = (int32_t)((uint32_t)s.Q[k] + (uint32_t)c.q[k]);
  }
  const int e1 = s.epoch_1ms, e19 = (s.epoch_1ms + 19) % 20;
  s.I_sum20 = (int32_t)((uint32_t)s.I_sum20 + ((uint32_t)c.i[1] - (uint32_t)s.I_buff[e1]));
  s.Q_sum20 = (int32_t)((uint32_t)s.Q_sum20 + ((uint32_t)c.q[1] - (uint32_t)s.Q_buff[e1]));
  s.I_buff[e1] = c.i[1];
  s.Q_buff[e1] = c.q[1];
  if ((s.I_buff[e1] > 0) != (s.I_buff[e19] > 0)) s.P_buff[e19]++;
  if ((s.epoch_1ms % s.len) == 0) dump_accum(s, fft, tw);
  est_cn0(s);
  bit_lock(s);
  bit_stuff(s, e);
  epoch(s);
  gnsscorr_sdr_feedback f = {};
  f.kill = s.state == kEmpty;
  f.carrier_nco = s.carrier_nco;
  f.code_nco = s.code_nco;
  if (s.bit_lock_pend && (s.epoch_1ms == 0)) {
    f.reset_1ms = 1;
    s.bit_lock_pend = 0;
  }
  if (s.frame_lock_pend) {
    f.reset_20ms = 1;
    s.frame_lock_pend = 0;
  }
  if (s.z_count_pend) {
    f.set_z_count = 1;
    f.z_count = (uint32_t)s.z_count;
    s.z_count_pend = 0;
  }
  s.navigate = s.converged ? 1 : 0;
  f.navigate = (uint32_t)s.navigate;
  *fb = f;
}

__global__ __launch_bounds__(64) void sdr_channel_kernel(
    int n_ch, int n_ms, const gnsscorr_sdr_corr* __restrict__ corr, Chan* __restrict__ chans,
    gnsscorr_sdr_feedback* __restrict__ fb, gnsscorr_sdr_feedback* __restrict__ fb_last,
    gnsscorr_sdr_subframe* __restrict__ ev, int max_ev, int32_t* __restrict__ n_ev,
    Twiddles tw) {
  // each thread's copy of its Channel object but the FFT buffer, in LDS (not
  // scratch: the serial channel code is a chain of dependent field accesses)
  __shared__ __attribute__((aligned(16))) unsigned char s_obj[64][offsetof(Chan, fft_buff)];
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= n_ch) return;
  Chan& g = chans[ch];
  Chan& s = *reinterpret_cast<Chan*>(s_obj[threadIdx.x]);   // fields before fft_buff only
  memcpy(&s, &g, offsetof(Chan, fft_buff));
  Events e = {ev, max_ev, n_ev, ch, 0};
  gnsscorr_sdr_feedback f = {};
  for (int m = 0; m < n_ms; m++) {
    e.ms = m;
    accum(s, g.fft_buff, tw, corr[(size_t)m * n_ch + ch], &f, e);
    if (fb) fb[(size_t)m * n_ch + ch] = f;
  }
  if (fb_last) fb_last[ch] = f;
  memcpy(&g, &s, offsetof(Chan, fft_buff));
}

// Device-resident closed loop: Correlator::Correlate (correlator.cpp:160-237)
// over n_packets packets with UpdateState, DumpAccum (:452-525) and the
// channel's Accum / ProcessFeedback (:530-555) at every dump -- the loop the
// reference runs per packet on the host, here without leaving the device.
// The schedule is the host's (gnsscorr_sdr_correlate): per packet at most 3
// segments, at most 2 dumps.
// One wavefront runs cpw channels.  Lane c (< cpw) owns channel ch0 + c: its
// correlator state, sums and Channel object sit in LDS and the lane runs the
// scalar work of its channel (bookkeeping, rotation, Channel::Accum,
// ProcessFeedback) -- the cpw channels' serial chains side by side in SIMD.
// Each Accum segment is done by the whole wave (sdrc::accum_wave), one channel
// after the other.  The scalar chain is latency bound, so lanes working for
// several channels at once is where the throughput comes from.
constexpr int kLoopMaxCpw = 16;
__global__ __launch_bounds__(64, 2) void sdr_track_kernel(
    const uint32_t* __restrict__ packets, int n_packets, int n_rx, int n_ch, int cpw,
    const int32_t* __restrict__ rx, gnsscorr_sdr_chan* __restrict__ states,
    gnsscorr_sdr_corr* __restrict__ corr, Chan* __restrict__ chans,
    gnsscorr_sdr_feedback* __restrict__ fb_last, gnsscorr_sdr_dump_rec* __restrict__ log,
    int log_per_ch, int32_t* __restrict__ n_log, int32_t* __restrict__ status,
    gnsscorr_sdr_subframe* __restrict__ ev, int max_ev, int32_t* __restrict__ n_ev,
    const uint32_t* __restrict__ carrier, const uint32_t* __restrict__ codebits, int saturate,
    Twiddles tw) {
  using namespace sdrc;
  __shared__ gnsscorr_sdr_chan s_st[kLoopMaxCpw];
  __shared__ gnsscorr_sdr_corr s_c[kLoopMaxCpw];
  __shared__ gnsscorr_sdr_accum_job s_job[kLoopMaxCpw];
  __shared__ int32_t s_rx[kLoopMaxCpw];
  // the Channel objects but their FFT buffers (those stay in HBM)
  __shared__ __attribute__((aligned(16))) unsigned char s_obj[kLoopMaxCpw][offsetof(Chan, fft_buff)];
  const int lane = threadIdx.x;
  const int ch0 = blockIdx.x * cpw;
  const int nc = min(cpw, n_ch - ch0);   // channels of this wave
  const bool own = lane < nc;
  const int ch = ch0 + (own ? lane : 0);
  Chan& cs = *reinterpret_cast<Chan*>(s_obj[own ? lane : 0]);   // fields before fft_buff only
  gnsscorr_sdr_feedback f = {};
  int32_t ndump = 0, stat = 0;
  if (own) {
    s_st[lane] = states[ch];
    s_c[lane] = corr[ch];
    memcpy(&cs, &chans[ch], offsetof(Chan, fft_buff));
    const int r = rx ? rx[ch] : 0;
    s_rx[lane] = r;
    if (r < 0 || r >= n_rx) stat = -1;
  }
  __syncthreads();
  Events e = {ev, max_ev, n_ev, ch, 0};
  for (int p = 0; p < n_packets; p++) {
    bool live = own && stat == 0 && s_st[lane].active;
    if (!__any(live)) break;   // a stopped or killed channel stays so
    int off = 0, left = kN, dumps = 0;
    for (int phase = 0; phase < 3; phase++) {
      bool dump = false;
      int samps = 0;
      if (own) {
        gnsscorr_sdr_accum_job j = {};
        if (live) {
          const gnsscorr_sdr_chan& s = s_st[lane];
          dump = dumps < 2 && s.rollover <= (uint32_t)left;
          samps = dump ? (int)s.rollover : left;
          j = make_job(s, 0, off, samps);
          if (samps > 0 && !job_in_range(j, 1)) {   // the host path returns EINVAL here
            stat = 1 + p;
            live = dump = false;
            samps = 0;
          }
        }
        j.samps = samps;
        s_job[lane] = j;
      }
      __syncthreads();
      for (int c = 0; c < nc; c++) {   // the segments, one channel after the other
        const gnsscorr_sdr_accum_job j = s_job[c];
        if (j.samps > 0) {
          const uint32_t* pkt = packets + ((size_t)p * n_rx + s_rx[c]) * kN;
          const gnsscorr_sdr_corr a = accum_wave(j, pkt, carrier, codebits, saturate);
          if (lane == c) {
            for (int k = 0; k < 3; k++) {
              s_c[c].i[k] = (int32_t)((uint32_t)s_c[c].i[k] + (uint32_t)a.i[k]);
              s_c[c].q[k] = (int32_t)((uint32_t)s_c[c].q[k] + (uint32_t)a.q[k]);
            }
          }
        }
      }
      if (live) {
        gnsscorr_sdr_chan* s = &s_st[lane];
        gnsscorr_sdr_corr* cc = &s_c[lane];
        if (samps > 0) update_state(s, samps);
        off += samps;
        left -= samps;
        if (dump) {
          rotate(s, cc);
          e.ms = p;
          accum(cs, chans[ch].fft_buff, tw, *cc, &f, e);
          if (ndump < log_per_ch) {
            gnsscorr_sdr_dump_rec& d = log[(size_t)ch * log_per_ch + ndump];
            d.packet = p;
            d.phase = phase;
            d.corr = *cc;
            d.fb = f;
          }
          after_feedback(s, cc, f);
          ndump++;
          dumps++;
        }
        if (!dump || !s->active) live = false;
      }
      __syncthreads();   // s_job is rewritten by the next phase
      if (!__any(live)) break;
    }
  }
  if (own) {
    states[ch] = s_st[lane];
    corr[ch] = s_c[lane];
    memcpy(&chans[ch], &cs, offsetof(Chan, fft_buff));
    if (fb_last && ndump > 0) fb_last[ch] = f;
    if (n_log) n_log[ch] = ndump;
    status[ch] = stat;
  }
}

Twiddles make_twiddles() {   // fft.cpp:121-149 for N = 512
  Twiddles t;
  const double pi = 3.14159265358979323846264338327;
  for (int k = 0; k < kFreqLockPoints / 2; k++) {
    const double ph = (-2 * pi * k) / kFreqLockPoints;
    const int16_t c = (int16_t)floor(16384 * cos(ph)), s = (int16_t)floor(16384 * sin(ph));
    t.w[k] = (uint32_t)(uint16_t)c | (uint32_t)(uint16_t)s << 16;
  }
  return t;
}

}  // namespace

static_assert(sizeof(gnsscorr_sdr_channel) == 2632, "gnsscorr_sdr_channel layout");

extern "C" int gnsscorr_sdr_channel_start(gnsscorr_sdr_channel* s, int chan, int sv,
                                          int acq_doppler, int corr_len) {
  if (!s) return GNSSCORR_EINVAL;
  // Channel::Channel (channel.cpp:31-57) then Start (:133-170)
  memset(s, 0, sizeof *s);
  s->chan = chan;
  clear(*s, s->fft_buff);
  s->sv = sv;
  s->code_nco = kCodeRate + acq_doppler * kCodeRate / kL1;
  s->carrier_nco = (double)(kIF + acq_doppler);
  s->dll[DX] = (float)(2.0 * acq_doppler * kCodeRate / kL1);
  s->pll[PW] = 0.0f;
  s->pll[PX] = (float)(2.0 * acq_doppler);
  s->pll[PZ] = (float)acq_doppler;
  s->len = corr_len == 20 ? 20 : 1;
  pll_w(*s, 18.0f);
  dll_w(*s, 1.0f);
  s->state = kNormal;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_channel_accum_dev(gnsscorr_sdr_corr_ctx* ctx, int n_ch, int n_ms,
                                              const gnsscorr_sdr_corr* d_corr,
                                              gnsscorr_sdr_channel* d_ch,
                                              gnsscorr_sdr_feedback* d_fb,
                                              gnsscorr_sdr_feedback* d_fb_last,
                                              gnsscorr_sdr_subframe* d_events, int max_events,
                                              int32_t* d_n_events) {
  if (!ctx || n_ch < 1 || n_ms < 0 || !d_corr || !d_ch || !d_n_events ||
      (max_events > 0 && !d_events)) {
    gnsscorr_set_error("gnsscorr_sdr_channel_accum_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  if (n_ms == 0) return GNSSCORR_OK;
  HIP_TRY(hipSetDevice(gnsscorr_sdr_corr_device(ctx)));
  hipStream_t s = (hipStream_t)gnsscorr_sdr_corr_stream(ctx);
  static const Twiddles tw = make_twiddles();
  hipLaunchKernelGGL(sdr_channel_kernel, dim3((n_ch + 63) / 64), dim3(64), 0, s, n_ch, n_ms,
                     d_corr, d_ch, d_fb, d_fb_last, d_events, max_events, d_n_events, tw);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_track_dev(gnsscorr_sdr_corr_ctx* ctx, const int16_t* d_packets,
                                      int n_packets, int n_rx, int n_ch, const int32_t* d_rx,
                                      gnsscorr_sdr_chan* d_states, gnsscorr_sdr_corr* d_corr,
                                      gnsscorr_sdr_channel* d_ch, gnsscorr_sdr_feedback* d_fb_last,
                                      gnsscorr_sdr_dump_rec* d_log, int log_per_ch,
                                      int32_t* d_n_log, int32_t* d_status,
                                      gnsscorr_sdr_subframe* d_events, int max_events,
                                      int32_t* d_n_events) {
  if (!ctx || n_packets < 0 || n_rx < 1 || n_ch < 0 || (n_packets > 0 && !d_packets) ||
      (n_ch > 0 && (!d_states || !d_corr || !d_ch || !d_status || !d_n_events)) ||
      log_per_ch < 0 || (log_per_ch > 0 && !d_log) || max_events < 0 ||
      (max_events > 0 && !d_events)) {
    gnsscorr_set_error("gnsscorr_sdr_track_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  if (n_ch == 0) return GNSSCORR_OK;
  HIP_TRY(hipSetDevice(gnsscorr_sdr_corr_device(ctx)));
  hipStream_t s = (hipStream_t)gnsscorr_sdr_corr_stream(ctx);
  const uint32_t *carrier, *codebits;
  int saturate;
  gnsscorr_sdr_corr_tables(ctx, &carrier, &codebits, &saturate);
  static const Twiddles tw = make_twiddles();
  // channels per wave: about two waves per SIMD for the whole launch (the
  // scalar chains are latency bound; a wave's lanes run cpw of them at once)
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                              gnsscorr_sdr_corr_device(ctx));
  int cpw = (n_ch + 8 * cus - 1) / (8 * cus);
  if (const char* ov = getenv("GNSSCORR_SDR_LOOP_CPW")) cpw = atoi(ov);
  cpw = cpw < 1 ? 1 : (cpw > kLoopMaxCpw ? kLoopMaxCpw : cpw);
  hipLaunchKernelGGL(sdr_track_kernel, dim3((n_ch + cpw - 1) / cpw), dim3(64), 0, s,
                     (const uint32_t*)d_packets, n_packets, n_rx, n_ch, cpw, d_rx, d_states,
                     d_corr, d_ch, d_fb_last, d_log, log_per_ch, d_n_log, d_status, d_events,
                     max_events, d_n_events, carrier, codebits, saturate, tw);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}
