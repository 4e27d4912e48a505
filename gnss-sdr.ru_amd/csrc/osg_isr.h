// osg_isr.h -- the OSGPS channel loops (gpsisr) as device code, shared by
// osg_isr_kernel (osg_loops.hip) and the fused closed-loop tail of
// osg_stream_kernel (track.hip).  See osg_loops.hip for the reference map:
// osgnss_next_step/src/isr/osgpsisr.c:360-768.
#ifndef GNSSCORR_OSG_ISR_H
#define GNSSCORR_OSG_ISR_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gnsscorr_internal.h"

namespace osgisr {

enum { kOff = 0, kAcq = 1, kConfirm = 2, kPullIn = 3, kTrack = 4 };
enum { iP = 0, qP = 1, iL = 2, qL = 3, iE = 4, qE = 5 };   // struct accum order

__host__ __device__ __forceinline__ int iabs(int v) { return v < 0 ? -v : v; }
template <typename T>
__host__ __device__ __forceinline__ int sgn(T x) { return x > 0 ? 1 : (x == 0 ? 0 : -1); }

// rss (osgpsisr.c:91-107): abs() of the long arguments is int abs
__device__ __forceinline__ int64_t rss(int64_t a, int64_t b) {
  const int64_t c = iabs((int)a), d = iabs((int)b);
  if (c == 0 && d == 0) return 0;
  return c > d ? (d >> 1) + c : (c >> 1) + d;
}

// fix_atan2 (osgpsisr.c:186-229), 1 rad = 16384
__device__ __forceinline__ int64_t fix_atan2(int64_t y, int64_t x) {
  const int64_t kPi2 = 25736, kPi = 51472;
  int64_t result = 0, n, n3;
  if (x == 0 && y == 0) return 0;
  if (x > 0 && x >= iabs((int)y)) {
    n = (y << 14) / x;
    n3 = ((((n * n) >> 14) * n) >> 13) / 9;
    result = n - n3;
  } else if (x <= 0 && -x >= iabs((int)y)) {
    n = (y << 14) / x;
    n3 = ((((n * n) >> 14) * n) >> 13) / 9;
    if (y > 0)
      result = n - n3 + kPi;
    else
      result = n - n3 - kPi;
  } else if (y > 0 && y > iabs((int)x)) {
    n = (x << 14) / y;
    n3 = ((((n * n) >> 14) * n) >> 13) / 9;
    result = kPi2 - n + n3;
  } else if (y < 0 && -y > iabs((int)x)) {
    n = (x << 14) / y;
    n3 = ((((n * n) >> 14) * n) >> 13) / 9;
    result = -n + n3 - kPi2;
  }
  return result;
}

// sqrt_newton (osgpsisr.c:150-171); the final `1/rslt == rslt-1` test never
// holds for rslt >= 1, so rslt is returned as is
__device__ __forceinline__ uint32_t sqrt_newton(int64_t L) {
  int64_t temp, div;
  uint32_t rslt = (uint32_t)L;
  if (L <= 0) return 0;
  if (L & 0xFFFF0000L)
    div = (L & 0xFF000000L) ? 0x3FFF : 0x3FF;
  else if (L & 0x0FF00L)
    div = 0x3F;
  else
    div = (L > 4) ? 0x7 : L;
  while (true) {
    temp = L / div + div;
    div = temp >> 1;
    div += temp & 1;
    if ((int64_t)rslt > div)
      rslt = (uint32_t)div;
    else
      return rslt;
  }
}

__device__ __forceinline__ uint32_t carrier_word(int64_t f, const gnsscorr_osg_loop_cfg& c) {
  return (uint32_t)(int64_t)((double)(f << c.carrier_shift) * c.clock_mult);
}
__device__ __forceinline__ uint32_t code_word(int64_t f, const gnsscorr_osg_loop_cfg& c) {
  return (uint32_t)(int64_t)((double)(f << c.code_shift) * c.clock_mult);
}

__device__ inline void ch_acq(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r, const gnsscorr_osg_loop_cfg& k) {
  if (iabs(c.n_freq) <= c.search_max_f) {
    const int64_t prompt_mag = rss(c.accum[iP], c.accum[qP]);
    if (prompt_mag > k.acq_thresh) {
      c.state = kConfirm;
      c.i_confirm = 0;
      c.n_thresh = 0;
      c.early_mag = c.prompt_mag = c.late_mag = 0;
    } else {
      r.slew = 1;            // ch_code_slew(ch, 1)
      c.codes += 1;
    }
    if (c.codes == c.search_max_prn_delay) {
      c.n_freq += c.del_freq;
      c.del_freq = -(c.del_freq + sgn(c.del_freq));
      c.carrier_freq = k.carrier_ref + c.carrier_cold_corr + k.d_freq * c.n_freq;
      r.carrier_incr = carrier_word(c.carrier_freq, k);
      c.codes = 0;
    }
  } else {
    c.n_freq = 0;
    c.del_freq = 1;
    c.carrier_freq = k.carrier_ref + c.carrier_cold_corr + k.d_freq * c.n_freq;
    r.carrier_incr = carrier_word(c.carrier_freq, k);
    c.codes = 0;
  }
  c.cn0 = 0;
}

__device__ inline void ch_confirm(gnsscorr_osg_loop& c, const gnsscorr_osg_loop_cfg& k) {
  const int64_t prompt_mag = rss(c.accum[iP], c.accum[qP]);
  const int64_t late_mag = rss(c.accum[iL], c.accum[qL]);
  const int64_t early_mag = rss(c.accum[iE], c.accum[qE]);
  c.early_mag += early_mag;
  c.prompt_mag += prompt_mag;
  c.late_mag += late_mag;
  if (prompt_mag > k.acq_thresh) c.n_thresh++;
  if (c.i_confirm == k.confirm_m) {
    if (c.n_thresh >= k.n_of_m_thresh) {
      c.state = kPullIn;
      c.cn0 = 0;
      c.ch_time = 0;
      c.ms_set = 0;
      c.old_carr_nco = c.old_code_nco = c.old_carr_error = c.old_code_error = 0;
      c.code_freq_basis = k.code_ref;
      c.carr_freq_basis = c.carrier_freq;
      c.sign_pos = c.prev_sign_pos = 0;
    } else {
      c.state = kAcq;
    }
  }
  c.i_confirm++;
}

// the FLL-assisted PLL and the DLL shared by pull-in and tracking
__device__ inline void loops(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r, const gnsscorr_osg_loop_cfg& k) {
  const int aiP = c.accum[iP], aqP = c.accum[qP], piP = c.prev_accum[iP], pqP = c.prev_accum[qP];
  if (aiP != 0 && aqP != 0 && piP != 0 && pqP != 0) {
    c.cross = (int64_t)(aiP * pqP - piP * aqP);                    // int arithmetic
    const int dt = aiP * piP + aqP * pqP;
    c.dot = (int64_t)(dt < 0 ? -(int64_t)dt : (int64_t)dt);       // labs
    c.cross = c.cross >> 8;
    c.dot = c.dot >> 8;
    c.freq_error = fix_atan2(c.cross, c.dot);
    c.carr_error = fix_atan2((int64_t)(aqP * sgn(aiP)), (int64_t)iabs(aiP)) / 2;
  } else {
    c.freq_error = 0;
    c.carr_error = c.old_carr_error;
  }
  c.carr_nco = c.old_carr_nco + ((int64_t)k.fll_i1 * c.carr_error -
                                 (int64_t)k.fll_i2 * c.old_carr_error -
                                 (int64_t)k.fll_i3 * c.freq_error) / 51472;
  c.old_carr_nco = c.carr_nco;
  c.old_carr_error = c.carr_error;
  c.carr_freq = c.carr_freq_basis + c.carr_nco;
  r.carrier_incr = carrier_word(c.carr_freq, k);                  // ch_carrier

  const int aiE = c.accum[iE], aqE = c.accum[qE], aiL = c.accum[iL], aqL = c.accum[qL];
  if (aiE != 0 && aqE != 0 && aiL != 0 && aqL != 0) {
    const int64_t e2 = aiE * aiE + aqE * aqE, l2 = aiL * aiL + aqL * aqL;   // int sums
    c.code_error = (int64_t)sqrt_newton(e2);
    c.code_error = c.code_error - (int64_t)sqrt_newton(l2);
    c.code_error = 8192 * c.code_error;
    c.code_error = c.code_error / (int64_t)((int)sqrt_newton(e2) + (int)sqrt_newton(l2));
  } else {
    c.code_error = c.old_code_error;
  }
  c.code_nco = c.old_code_nco +
               (((int64_t)(k.dll_i1 + 1) * c.code_error - (int64_t)k.dll_i2 * c.old_code_error) /
                8192);
  c.old_code_nco = c.code_nco;
  c.old_code_error = c.code_error;
  c.code_freq = c.code_freq_basis - c.code_nco;
  r.code_incr = code_word(c.code_freq, k);                        // ch_code
}

__device__ inline void ch_pull_in(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r,
                           const gnsscorr_osg_loop_cfg& k) {
  loops(c, r, k);
  const int aiP = c.accum[iP], piP = c.prev_accum[iP];
  if (sgn(aiP) == -sgn(piP)) {
    c.prev_sign_pos = c.sign_pos;
    c.sign_pos = (int32_t)c.ch_time;
    if ((c.sign_pos - c.prev_sign_pos) > 19)
      c.sign_count++;
    else
      c.sign_count = 0;
  }
  c.ms_count++;
  if ((sgn(aiP) == -1 && (c.ms_sign & 0xfffff) == 0x00000) ||
      (sgn(aiP) == 1 && (c.ms_sign & 0xfffff) == 0xfffff)) {
    if (sgn(aiP) == -sgn(piP)) {
      c.ms_count = 0;
      r.epoch_load = 0x1;    // ch_epoch_load(ch, 0x1)
      c.ms_set = 1;
    }
  }
  c.ms_sign = c.ms_sign << 1;
  if (aiP < 0) c.ms_sign = c.ms_sign | 0x1;
  c.ms_count = c.ms_count % 20;
  c.ch_time++;
  if (c.sign_count > 30 && c.ms_set) c.state = kTrack;
  if (c.ch_time == 3000) {
    c.del_freq = 1;
    c.n_freq = 0;
    r.carrier_incr = carrier_word(k.carrier_ref, k);
    r.code_incr = code_word(k.code_ref, k);
    c.codes = 0;
    c.ch_time = 0;
    c.state = kAcq;
  }
}

__device__ inline void ch_track(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r, const gnsscorr_osg_loop_cfg& k) {
  loops(c, r, k);
  c.ms_count = (c.ms_count + 1) % 20;
  if (c.ms_count == 19) c.bit = c.accum[iP] > 0 ? 1 : 0;   // bsign
}


// One interrupt of one channel (gpsisr :360-404): the register bookkeeping of
// the call that just ran, then, if the channel dumped, the accumulators and
// the channel's state machine.  r: the channel's command words (in/out), c:
// its loop state (in/out), q: the call's result.
__device__ __forceinline__ void isr_step(const gnsscorr_osg_loop_cfg& k, gnsscorr_osg_loop& c,
                                         gnsscorr_nco_cmd& r, const gnsscorr_track_result& q) {
  // register bookkeeping of the call that just ran (osg_legacy.c Sim_GP2021_int)
  if (r.epoch_load != -1) r.epoch_load = -1;
  if (q.n_dumps > 0) {
    r.slew = 0;
    // gpsisr :366-378 -- prev_accum = accum; accum = from_gps(REG_read ...)
    for (int i = 0; i < 6; i++) c.prev_accum[i] = c.accum[i];
    c.accum[iE] = (int16_t)q.dump[4];
    c.accum[qE] = (int16_t)q.dump[5];
    c.accum[iP] = (int16_t)q.dump[2];
    c.accum[qP] = (int16_t)q.dump[3];
    c.accum[iL] = (int16_t)q.dump[0];
    c.accum[qL] = (int16_t)q.dump[1];
    switch (c.state) {
      case kOff: c.exited = 1; break;
      case kAcq: ch_acq(c, r, k); break;
      case kConfirm: ch_confirm(c, k); break;
      case kPullIn: ch_pull_in(c, r, k); break;
      case kTrack: ch_track(c, r, k); break;
      default: break;
    }
  }
}

}  // namespace osgisr
#endif
