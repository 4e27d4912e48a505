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
#include <stdlib.h>
#include "gnsscorr_internal.h"
#include "osg_isr.h"

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      gnsscorr_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                     \
      return GNSSCORR_EDEVICE;                                                          \
    }                                                                                   \
  } while (0)

using namespace osgisr;

namespace {

__global__ __launch_bounds__(256) void osg_isr_kernel(int n_ch, gnsscorr_osg_loop_cfg k,
                                                      gnsscorr_osg_loop* __restrict__ loops_,
                                                      gnsscorr_nco_cmd* __restrict__ cmds,
                                                      const gnsscorr_track_result* __restrict__ res,
                                                      gnsscorr_osg_loop* __restrict__ hist) {
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= n_ch) return;
  gnsscorr_nco_cmd r = cmds[ch];
  gnsscorr_osg_loop c = loops_[ch];
  osgisr::isr_step(k, c, r, res[ch]);
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
  // Two launches per call (the open-loop correlator, then osg_isr_kernel with 64
  // channels per wave) unless GNSSCORR_OSG_FUSED=1: the fused launch (every call and
  // every channel's gpsisr step in osg_stream_kernel, gpsisr on one lane of each
  // channel's wave) is byte-identical but, since the open-loop kernel's round-6
  // set-up work, 6 % slower (0.104 against 0.098 ms per 12 288-channel call: 165
  // VGPRs and no LO read-ahead, profiles/r6/closed_loop_fused_ab_r6z.log)
  const char* fe = getenv("GNSSCORR_OSG_FUSED");
  if (fe && fe[0] == '1') {
    // every call and every channel's gpsisr step in ONE launch
    const int rf = gnsscorr_track_dev_isr(ctx, d_if, stream_stride, nsamp, n_calls, d_cmds,
                                          d_res_hist, n_ch, cfg, d_loops, d_loop_hist);
    if (rf != GNSSCORR_TRACK_NOT_FUSED) return rf;
  }
  for (int k = 0; k < n_calls; k++) {
    gnsscorr_track_result* r = d_res_hist + (size_t)k * n_ch;
    const int64_t tic = gnsscorr_track_next_tic(ctx, nsamp);
    gnsscorr_osg_loop* h = d_loop_hist ? d_loop_hist + (size_t)k * n_ch : nullptr;
    int rc = gnsscorr_track_dev(ctx, d_if + k * bytes_per_call, stream_stride, nsamp, d_cmds, r,
                                nullptr, tic);
    if (rc) return rc;
    // one wave per workgroup: the per-channel state machine is a serial chain
    // (64-bit divides in the discriminators), so spread it over as many CUs as
    // possible instead of stacking four waves on a SIMD
    hipLaunchKernelGGL(osg_isr_kernel, dim3((n_ch + 63) / 64), dim3(64), 0, s, n_ch, *cfg,
                       d_loops, d_cmds, r, h);
    HIP_TRY(hipGetLastError());
  }
  return GNSSCORR_OK;
}
