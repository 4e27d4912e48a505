// osg_loops.hip -- the OSGPS channel loops (gpsisr) on gfx950.
//
// Reference: POSTPROCESSING_RECEIVERS/osgnss_next_step/src/isr/osgpsisr.c
//   gpsisr       :360-404  read the accumulators of every channel that dumped,
//                          then run its state
//   ch_acq       :418-457  serial code / Doppler search (half-chip slews)
//   ch_confirm   :473-520  n-of-m confirmation
//   ch_pull_in   :535-680  FLL-assisted PLL + DLL, bit-edge / ms-counter sync
//   ch_track     :700-768  the same loops, ms counter, data bit
//   rss :91-107, fix_atan2 :186-229, sqrt_newton :150-171 (fixed point helpers)
// Register writes follow gp2021/gp2021.c:75-130 (ch_carrier, ch_code,
// ch_code_slew, ch_epoch_load) and the legacy shim's REG_write handling
// (osg_legacy.c): carrier word = (uint32)((f << (32 - 30)) * 5.0), code word =
// (uint32)((f << (32 - 29)) * 5.0), an epoch load is consumed by the call that
// sees it, a slew lasts until the next dump.
//
// One thread per channel; `long` is int64 as in the reference's LP64 build,
// `abs()` of a long argument truncates to int first, `short` accumulators come
// from from_gps()'s int16 truncation.  CHANNEL_OFF with a dump makes the
// reference exit(0); here the channel is flagged (loop.exited) and left alone.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
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

__device__ void ch_acq(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r, const gnsscorr_osg_loop_cfg& k) {
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

__device__ void ch_confirm(gnsscorr_osg_loop& c, const gnsscorr_osg_loop_cfg& k) {
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
__device__ void loops(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r, const gnsscorr_osg_loop_cfg& k) {
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

__device__ void ch_pull_in(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r,
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

__device__ void ch_track(gnsscorr_osg_loop& c, gnsscorr_nco_cmd& r, const gnsscorr_osg_loop_cfg& k) {
  loops(c, r, k);
  c.ms_count = (c.ms_count + 1) % 20;
  if (c.ms_count == 19) c.bit = c.accum[iP] > 0 ? 1 : 0;   // bsign
}

__global__ __launch_bounds__(256) void osg_isr_kernel(int n_ch, gnsscorr_osg_loop_cfg k,
                                                      gnsscorr_osg_loop* __restrict__ loops_,
                                                      gnsscorr_nco_cmd* __restrict__ cmds,
                                                      const gnsscorr_track_result* __restrict__ res,
                                                      gnsscorr_osg_loop* __restrict__ hist) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= n_ch) return;
  gnsscorr_nco_cmd r = cmds[ch];
  const gnsscorr_track_result& q = res[ch];
  // register bookkeeping of the call that just ran (osg_legacy.c Sim_GP2021_int)
  if (r.epoch_load != -1) r.epoch_load = -1;
  gnsscorr_osg_loop c = loops_[ch];
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
  loops_[ch] = c;
  cmds[ch] = r;
  if (hist) hist[ch] = c;
}

}  // namespace

extern "C" void gnsscorr_osg_loop_cfg_init(gnsscorr_osg_loop_cfg* cfg, double samp_rate,
                                           double gps_if, double clock_mult, int carrier_nco_bits,
                                           int code_nco_bits, double bin_width, long bnp, long bnf,
                                           long bnd, long fll_t_ms, long dll_t_ms, int acq_thresh) {
  memset(cfg, 0, sizeof *cfg);
  // correlator.c:110-121
  const double cdelta = clock_mult * samp_rate / pow(2.0, carrier_nco_bits);
  const double kdelta = clock_mult * samp_rate / pow(2.0, code_nco_bits);
  cfg->code_ref = (int64_t)(1023000 / kdelta);
  cfg->carrier_ref = (int64_t)(gps_if / cdelta);
  cfg->d_freq = (int64_t)((int)bin_width / cdelta);
  // osgpsisr.c:253-266 calc_FLL_assisted_PLL_filter_loop_coefs
  const double wnp = bnp / 0.53, wnf = bnf / 0.25, T = (double)fll_t_ms / 1000, a2 = 1.414;
  const double k1 = T * (wnp * wnp) + a2 * wnp, k2 = a2 * wnp, k3 = T * wnf;
  // :281-286 convert_... (1 << bits) / (SAMP_RATE * SYSTEM_CLOCK_MULTIPLIER)
  const double cs = (double)(1 << carrier_nco_bits) / (samp_rate * clock_mult);
  cfg->fll_i1 = (int)(k1 * cs);
  cfg->fll_i2 = (int)(k2 * cs);
  cfg->fll_i3 = (int)(k3 * cs);
  // :306-318 calc_DLL_loop_filter_coefs, :325-330 convert
  const double w = bnd / 0.53, Td = (double)dll_t_ms / 1000;
  const double d1 = Td * (w * w) + a2 * w, d2 = a2 * w;
  const double ks = (double)(1 << code_nco_bits) / (samp_rate * clock_mult);
  cfg->dll_i1 = (int)(d1 * ks);
  cfg->dll_i2 = (int)(d2 * ks);
  cfg->acq_thresh = acq_thresh;
  cfg->confirm_m = 3;        // CONFIRM_M (globals.h:8)
  cfg->n_of_m_thresh = 2;    // N_OF_M_THRESH (globals.h:9)
  cfg->carrier_shift = 32 - carrier_nco_bits;
  cfg->code_shift = 32 - code_nco_bits;
  cfg->clock_mult = clock_mult;
}

extern "C" void gnsscorr_osg_loop_reset(const gnsscorr_osg_loop_cfg* cfg, int n_ch,
                                        const int32_t* prns, gnsscorr_osg_loop* loops,
                                        gnsscorr_nco_cmd* cmds) {
  for (int ch = 0; ch < n_ch; ch++) {
    gnsscorr_osg_loop& c = loops[ch];
    memset(&c, 0, sizeof c);
    c.state = kAcq;
    c.carrier_cold_corr = 0;
    c.del_freq = 1;
    c.n_freq = 0;
    c.search_max_prn_delay = 2045;
    c.search_max_f = 5;
    c.ms_set = 0;
    gnsscorr_nco_cmd& r = cmds[ch];
    memset(&r, 0, sizeof r);
    r.prn = prns ? prns[ch] : 0;
    r.carrier_incr = (uint32_t)(int64_t)((double)(cfg->carrier_ref << cfg->carrier_shift) *
                                         cfg->clock_mult);
    r.code_incr = (uint32_t)(int64_t)((double)(cfg->code_ref << cfg->code_shift) * cfg->clock_mult);
    r.slew = 0;
    r.epoch_load = 0;   // REG_write[(ch<<3)+7] is 0 at start: the first call loads epoch 0
    r.stream = 0;
  }
}

extern "C" int gnsscorr_osg_isr_dev(gnsscorr_track_ctx* ctx, const gnsscorr_osg_loop_cfg* cfg,
                                    int n_ch, gnsscorr_osg_loop* d_loops, gnsscorr_nco_cmd* d_cmds,
                                    const gnsscorr_track_result* d_res) {
  if (!ctx || !cfg || n_ch < 1 || !d_loops || !d_cmds || !d_res) {
    gnsscorr_set_error("gnsscorr_osg_isr_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  hipStream_t s = (hipStream_t)gnsscorr_track_stream(ctx);
  hipLaunchKernelGGL(osg_isr_kernel, dim3((n_ch + 63) / 64), dim3(64), 0, s, n_ch, *cfg,
                     d_loops, d_cmds, d_res, (gnsscorr_osg_loop*)nullptr);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_osg_closed_loop_dev(gnsscorr_track_ctx* ctx,
                                            const gnsscorr_osg_loop_cfg* cfg, const int8_t* d_if,
                                            int64_t stream_stride, int64_t nsamp, int n_calls,
                                            int n_ch, gnsscorr_osg_loop* d_loops,
                                            gnsscorr_nco_cmd* d_cmds,
                                            gnsscorr_track_result* d_res_hist,
                                            gnsscorr_osg_loop* d_loop_hist) {
  if (!ctx || !cfg || !d_if || n_calls < 1 || n_ch < 1 || !d_loops || !d_cmds || !d_res_hist) {
    gnsscorr_set_error("gnsscorr_osg_closed_loop_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  hipStream_t s = (hipStream_t)gnsscorr_track_stream(ctx);
  const int64_t bytes_per_call = gnsscorr_track_if_bytes(ctx, nsamp);
  for (int k = 0; k < n_calls; k++) {
    gnsscorr_track_result* r = d_res_hist + (size_t)k * n_ch;
    const int64_t tic = gnsscorr_track_next_tic(ctx, nsamp);
    int rc = gnsscorr_track_dev(ctx, d_if + k * bytes_per_call, stream_stride, nsamp, d_cmds, r,
                                nullptr, tic);
    if (rc) return rc;
    // one wave per workgroup: the per-channel state machine is a serial chain
    // (64-bit divides in the discriminators), so spread it over as many CUs as
    // possible instead of stacking four waves on a SIMD
    hipLaunchKernelGGL(osg_isr_kernel, dim3((n_ch + 63) / 64), dim3(64), 0, s, n_ch, *cfg,
                       d_loops, d_cmds, r, d_loop_hist ? d_loop_hist + (size_t)k * n_ch : nullptr);
    HIP_TRY(hipGetLastError());
  }
  return GNSSCORR_OK;
}
