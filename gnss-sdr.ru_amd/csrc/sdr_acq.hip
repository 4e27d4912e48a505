// sdr_acq.hip -- GPS-SDR int16 strong acquisition on gfx950, bit-exact.
//
// Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER
//   Acquisition::doPrepIF   objects/acquisition.cpp:191-236 (1 ms, type 0)
//   Acquisition::doAcqStrong objects/acquisition.cpp:244-301
//   FFT (radix-2 DIT, Q14 twiddles, per-rank 1/2 scaling) objects/fft.cpp:114-245, 403-441
//   x86_cmulsc / sse_cmulsc  simd/x86.cpp:184-214, simd/sse.cpp:646-729
//   x86_cmag, x86_max        simd/x86.cpp:250-288
//
// Work decomposition (one 1-ms 2048-sample CPX buffer per record):
//   sdr_prep_kernel    one workgroup per (record, 250 Hz sub-bin j):
//                      wipe-off (cmulsc, shift 14) written straight into
//                      bit-reversed LDS positions, 11 unscaled DIT ranks,
//                      spectrum row X[rec][j][2048] to HBM (natural order).
//   sdr_strong_kernel  one workgroup per (record, sv, row) with row =
//                      (lcv - lmin)*4 + lcv2: reads X[rec][lcv2] circularly
//                      from offset lcv (the reference's baseband_rows[...]
//                      [100+lcv] rotation), cmulsc by the PRN spectrum (shift
//                      10), bit-reversed into LDS, 11 inverse ranks with the
//                      R2 scaling mask, |.|^2 as int32 and a first-index max.
//   sdr_select_kernel  per (record, sv): the strict-greater scan over rows in
//                      (lcv, lcv2) order of doAcqStrong.
// All arithmetic is the reference's int16/int32 with its wrap points; butterflies
// of one rank are independent, so only the rank order has to be kept.
// Roofline: integer VALU + LDS (each rank = 2048 LDS reads/writes of 4 B).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
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

constexpr int kN = 2048;
constexpr int kM = 11;
constexpr int kThreads = 256;
constexpr int kMaxLcv = 100;      // baseband_rows padding (acquisition.cpp:229-233)
constexpr uint32_t kR2 = (1u << 7) | (1u << 9);   // R2 = {0 x7, 1, 0, 1, 0, ...} (ranks 0..10)

__device__ __forceinline__ int16_t lo16(uint32_t v) { return (int16_t)(v & 0xFFFFu); }
__device__ __forceinline__ int16_t hi16(uint32_t v) { return (int16_t)(v >> 16); }
__device__ __forceinline__ uint32_t pack(int16_t i, int16_t q) {
  return (uint32_t)(uint16_t)i | ((uint32_t)(uint16_t)q << 16);
}
__device__ __forceinline__ int16_t sat16(int32_t v) {
  return (int16_t)(v > 32767 ? 32767 : (v < -32768 ? -32768 : v));
}

// C = (A*B + 2^(s-1)) >> s, complex, wrapped (x86) or saturated (sse packssdw)
__device__ __forceinline__ uint32_t cmulsc(uint32_t a, uint32_t b, int shift, bool sat) {
  const int32_t ai = lo16(a), aq = hi16(a), bi = lo16(b), bq = hi16(b);
  const int32_t rnd = 1 << (shift - 1);
  const int32_t ti = (ai * bi - aq * bq + rnd) >> shift;
  const int32_t tq = (ai * bq + aq * bi + rnd) >> shift;
  return sat ? pack(sat16(ti), sat16(tq)) : pack((int16_t)ti, (int16_t)tq);
}

__device__ __forceinline__ int brev11(int k) { return (int)(__brev((uint32_t)k) >> 21); }

// 11 radix-2 DIT ranks in LDS (fft.cpp:156-180 with the rank/bfly loops of :314-334)
// tw: packed (c, s) Q14 twiddles, 1024 entries, forward or inverse
__device__ void dit_ranks(uint32_t* x, const uint32_t* tw, uint32_t scale_mask) {
  for (int r = 0; r < kM; r++) {
    const bool scale = (scale_mask >> r) & 1u;
#pragma unroll
    for (int u = 0; u < (kN / 2) / kThreads; u++) {
      const int t = threadIdx.x + u * kThreads;
      const int j = t & ((1 << r) - 1);
      const int a = ((t >> r) << (r + 1)) + j;
      const int b = a + (1 << r);
      const uint32_t w = tw[j << (kM - 1 - r)];
      const int32_t wi = lo16(w), wq = hi16(w);
      const uint32_t A = x[a], B = x[b];
      int16_t ai = lo16(A), aq = hi16(A), bi0 = lo16(B), bq0 = hi16(B);
      if (scale) { ai >>= 1; aq >>= 1; bi0 >>= 1; bq0 >>= 1; }
      int32_t bi = (int32_t)bi0 * wi - (int32_t)bq0 * wq;
      int32_t bq = (int32_t)bi0 * wq + (int32_t)bq0 * wi;
      bi = (bi + 8192) >> 14;
      bq = (bq + 8192) >> 14;
      x[b] = pack((int16_t)(ai - (int16_t)bi), (int16_t)(aq - (int16_t)bq));
      x[a] = pack((int16_t)(ai + (int16_t)bi), (int16_t)(aq + (int16_t)bq));
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kThreads) void sdr_prep_kernel(
    const uint32_t* __restrict__ buff, const uint32_t* __restrict__ wipe,
    const uint32_t* __restrict__ tw_fwd, uint32_t* __restrict__ X, int saturate) {
  __shared__ uint32_t x[kN];
  __shared__ uint32_t tw[kN / 2];
  const int rec = blockIdx.x >> 2, j = blockIdx.x & 3;
  const uint32_t* src = buff + (size_t)rec * kN;
  const uint32_t* wp = wipe + (size_t)j * kN;
  for (int k = threadIdx.x; k < kN / 2; k += kThreads) tw[k] = tw_fwd[k];
  for (int k = threadIdx.x; k < kN; k += kThreads)
    x[brev11(k)] = cmulsc(src[k], wp[k], 14, saturate != 0);   // + doShuffle
  __syncthreads();
  dit_ranks(x, tw, 0u);                                         // R1: no scaling
  uint32_t* dst = X + ((size_t)rec * 4 + j) * kN;
  for (int k = threadIdx.x; k < kN; k += kThreads) dst[k] = x[k];
}

// per-row result: (magnitude, index) of x86_cmag + x86_max
__global__ __launch_bounds__(kThreads) void sdr_strong_kernel(
    const uint32_t* __restrict__ X, const uint32_t* __restrict__ codes,
    const uint32_t* __restrict__ tw_inv, const int32_t* __restrict__ svs, int n_sv, int lmin,
    int n_rows, int saturate, int2* __restrict__ row_out) {
  __shared__ uint32_t x[kN];
  __shared__ uint32_t tw[kN / 2];
  __shared__ int2 red[kThreads / 64];
  const int row = blockIdx.x % n_rows;
  const int s = (blockIdx.x / n_rows) % n_sv;
  const int rec = blockIdx.x / (n_rows * n_sv);
  const int lcv = lmin + (row >> 2), lcv2 = row & 3;
  const uint32_t* xr = X + ((size_t)rec * 4 + lcv2) * kN;
  const uint32_t* cr = codes + (size_t)svs[s] * kN;
  for (int k = threadIdx.x; k < kN / 2; k += kThreads) tw[k] = tw_inv[k];
  for (int k = threadIdx.x; k < kN; k += kThreads)
    x[brev11(k)] = cmulsc(xr[(k + lcv) & (kN - 1)], cr[k], 10, saturate != 0);
  __syncthreads();
  dit_ranks(x, tw, kR2);
  // x86_cmag (int32 wrap) + x86_max (first index of the strict maximum, > 0)
  int32_t best = 0, idx = 0;
  for (int k = threadIdx.x; k < kN; k += kThreads) {
    const uint32_t v = x[k];
    const int32_t i = lo16(v), q = hi16(v);
    const int32_t p = (int32_t)((uint32_t)(i * i) + (uint32_t)(q * q));
    if (p > best) { best = p; idx = k; }
  }
  // reduce: larger magnitude wins, equal magnitude -> smaller index
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int32_t ob = __shfl_xor(best, o, 64), oi = __shfl_xor(idx, o, 64);
    if (ob > best || (ob == best && oi < idx)) { best = ob; idx = oi; }
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_int2(best, idx);
  __syncthreads();
  if (threadIdx.x == 0) {
    int2 r = red[0];
    for (int w = 1; w < kThreads / 64; w++) {
      const int2 o = red[w];
      if (o.x > r.x || (o.x == r.x && o.y < r.y)) r = o;
    }
    if (r.x <= 0) r = make_int2(0, 0);
    row_out[blockIdx.x] = r;
  }
}

__global__ void sdr_select_kernel(const int2* __restrict__ row_out, const int32_t* __restrict__ svs,
                                  int n_sv, int n_rec, int lmin, int n_rows,
                                  gnsscorr_sdr_acq_result* __restrict__ res) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_rec * n_sv) return;
  const int2* rr = row_out + (size_t)g * n_rows;
  gnsscorr_sdr_acq_result r = {};
  r.sv = svs[g % n_sv];
  int32_t mag = 0;
  for (int row = 0; row < n_rows; row++) {   // doAcqStrong: lcv outer, lcv2 inner, strict >
    const int2 v = rr[row];
    if (v.x > mag) {
      mag = v.x;
      r.code_phase = kN - v.y;
      r.doppler = (lmin + (row >> 2)) * 1000 + (row & 3) * 250;
      r.magnitude = (uint32_t)v.x;
      r.row = row;
    }
  }
  r.success = r.magnitude > 0u;   // THRESH_STRONG = 0 (config.h:72)
  res[g] = r;
}

}  // namespace

// ============================================================================
// host side
// ============================================================================
struct gnsscorr_sdr_acq_ctx {
  gnsscorr_sdr_acq_cfg cfg;
  hipStream_t stream = nullptr;
  uint32_t *d_wipe = nullptr, *d_codes = nullptr, *d_twf = nullptr, *d_twi = nullptr;
  uint32_t *d_X = nullptr, *d_buff = nullptr;
  int32_t* d_svs = nullptr;
  int2* d_rows = nullptr;
  gnsscorr_sdr_acq_result* d_res = nullptr;
  size_t cap_rec = 0, cap_rows = 0, cap_sv = 0;
};

extern "C" int gnsscorr_sdr_acq_destroy(gnsscorr_sdr_acq_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* ps[] = {c->d_wipe, c->d_codes, c->d_twf, c->d_twi, c->d_X,
                c->d_buff, c->d_svs,   c->d_rows, c->d_res};
  for (void* p : ps) (void)hipFree(p);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_acq_create(gnsscorr_sdr_acq_ctx** out, const gnsscorr_sdr_acq_cfg* cfg) {
  if (!out || !cfg) return GNSSCORR_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gnsscorr_set_error("gnsscorr_sdr_acq_create: no HIP device");
    return GNSSCORR_ENODEV;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    gnsscorr_set_error("gnsscorr_sdr_acq_create: device %d out of range", cfg->device);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(cfg->device));
  auto* c = new gnsscorr_sdr_acq_ctx();
  c->cfg = *cfg;
  // host tables: wipe-offs (sine_gen, misc.cpp:95-115), Q14 twiddles (fft.cpp:114-147),
  // PRN spectra (gen_fft_codes.m)
  uint32_t* h = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)(4 * kN + 51 * kN + kN));
  int16_t* tmp = (int16_t*)malloc(sizeof(int16_t) * 2 * (size_t)51 * kN);
  int rc = (h && tmp) ? GNSSCORR_OK : GNSSCORR_ENOMEM;
  if (!rc) {
    for (int j = 0; j < 4; j++) {
      gnsscorr_sdr_sine_gen(tmp, -cfg->fif - 250.0 * j, 2048000.0, kN);
      memcpy(h + (size_t)j * kN, tmp, sizeof(uint32_t) * kN);
    }
    gnsscorr_sdr_prn_codes(tmp);
    memcpy(h + 4 * kN, tmp, sizeof(uint32_t) * 51 * kN);
    gnsscorr_sdr_twiddles((int16_t*)(h + 55 * kN), (int16_t*)(h + 55 * kN + kN / 2));
  }
  hipError_t e = hipSuccess;
  if (!rc) {
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->d_wipe, sizeof(uint32_t) * 4 * kN);
    if (e == hipSuccess) e = hipMalloc(&c->d_codes, sizeof(uint32_t) * 51 * kN);
    if (e == hipSuccess) e = hipMalloc(&c->d_twf, sizeof(uint32_t) * kN / 2);
    if (e == hipSuccess) e = hipMalloc(&c->d_twi, sizeof(uint32_t) * kN / 2);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_wipe, h, sizeof(uint32_t) * 4 * kN, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_codes, h + 4 * kN, sizeof(uint32_t) * 51 * kN, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_twf, h + 55 * kN, sizeof(uint32_t) * kN / 2, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_twi, h + 55 * kN + kN / 2, sizeof(uint32_t) * kN / 2,
                    hipMemcpyHostToDevice);
  }
  free(h);
  free(tmp);
  if (rc || e != hipSuccess) {
    if (e != hipSuccess) gnsscorr_set_error("gnsscorr_sdr_acq_create: %s", hipGetErrorString(e));
    gnsscorr_sdr_acq_destroy(c);
    return rc ? rc : GNSSCORR_EDEVICE;
  }
  *out = c;
  return GNSSCORR_OK;
}

static int grow(void** p, size_t* cap, size_t need, size_t elem) {
  if (need <= *cap) return GNSSCORR_OK;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, need * elem));
  *cap = need;
  return GNSSCORR_OK;
}

static int check_range(int n_rec, int n_sv, int doppmin, int doppmax) {
  const int lmin = doppmin / 1000, lmax = doppmax / 1000;   // C truncation, as the reference
  if (n_rec < 1 || n_sv < 1 || lmax <= lmin || lmin < -kMaxLcv || lmax > kMaxLcv + 1) {
    gnsscorr_set_error("gnsscorr_sdr_acq_strong: need n_rec>=1, n_sv>=1 and "
                       "-100 <= doppmin/1000 < doppmax/1000 <= 101 (the +-100-bin row padding)");
    return GNSSCORR_EINVAL;
  }
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_acq_strong_dev(gnsscorr_sdr_acq_ctx* c, const int16_t* d_buff,
                                           int n_rec, int n_sv, const int32_t* d_svs,
                                           int doppmin, int doppmax,
                                           gnsscorr_sdr_acq_result* d_res) {
  if (!c || !d_buff || !d_svs || !d_res) return GNSSCORR_EINVAL;
  int rc = check_range(n_rec, n_sv, doppmin, doppmax);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->cfg.device));
  const int lmin = doppmin / 1000, n_rows = 4 * (doppmax / 1000 - lmin);
  if ((rc = grow((void**)&c->d_X, &c->cap_rec, (size_t)n_rec, sizeof(uint32_t) * 4 * kN)))
    return rc;
  if ((rc = grow((void**)&c->d_rows, &c->cap_rows, (size_t)n_rec * n_sv * n_rows, sizeof(int2))))
    return rc;
  hipLaunchKernelGGL(sdr_prep_kernel, dim3(4 * n_rec), dim3(kThreads), 0, c->stream,
                     (const uint32_t*)d_buff, c->d_wipe, c->d_twf, c->d_X, c->cfg.saturate);
  hipLaunchKernelGGL(sdr_strong_kernel, dim3(n_rec * n_sv * n_rows), dim3(kThreads), 0, c->stream,
                     c->d_X, c->d_codes, c->d_twi, d_svs, n_sv, lmin, n_rows, c->cfg.saturate,
                     c->d_rows);
  const int G = n_rec * n_sv;
  hipLaunchKernelGGL(sdr_select_kernel, dim3((G + 63) / 64), dim3(64), 0, c->stream, c->d_rows,
                     d_svs, n_sv, n_rec, lmin, n_rows, d_res);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_acq_strong(gnsscorr_sdr_acq_ctx* c, const int16_t* h_buff, int n_rec,
                                       int n_sv, const int32_t* h_svs, int doppmin, int doppmax,
                                       gnsscorr_sdr_acq_result* h_res) {
  if (!c || !h_buff || !h_svs || !h_res) return GNSSCORR_EINVAL;
  int rc = check_range(n_rec, n_sv, doppmin, doppmax);
  if (rc) return rc;
  for (int k = 0; k < n_sv; k++)
    if (h_svs[k] < 0 || h_svs[k] >= 32) {   // fft_codes[] covers MAX_SV = 32 (config.h:52)
      gnsscorr_set_error("gnsscorr_sdr_acq_strong: sv %d out of range 0..31", h_svs[k]);
      return GNSSCORR_EINVAL;
    }
  HIP_TRY(hipSetDevice(c->cfg.device));
  static_assert(sizeof(gnsscorr_sdr_acq_result) == 24, "result layout");
  // staging buffers sized to this call
  size_t cap_b = 0, cap_s = 0, cap_r = 0;
  int16_t* d_b = nullptr;
  int32_t* d_s = nullptr;
  gnsscorr_sdr_acq_result* d_r = nullptr;
  auto cleanup = [&]() {
    (void)hipFree(d_b);
    (void)hipFree(d_s);
    (void)hipFree(d_r);
  };
  if ((rc = grow((void**)&d_b, &cap_b, (size_t)n_rec * kN, sizeof(uint32_t))) ||
      (rc = grow((void**)&d_s, &cap_s, (size_t)n_sv, sizeof(int32_t))) ||
      (rc = grow((void**)&d_r, &cap_r, (size_t)n_rec * n_sv, sizeof(gnsscorr_sdr_acq_result)))) {
    cleanup();
    return rc;
  }
  hipError_t e = hipMemcpyAsync(d_b, h_buff, sizeof(uint32_t) * (size_t)n_rec * kN,
                                hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_s, h_svs, sizeof(int32_t) * n_sv, hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) {
    cleanup();
    gnsscorr_set_error("gnsscorr_sdr_acq_strong: %s", hipGetErrorString(e));
    return GNSSCORR_EDEVICE;
  }
  rc = gnsscorr_sdr_acq_strong_dev(c, d_b, n_rec, n_sv, d_s, doppmin, doppmax, d_r);
  if (!rc) {
    e = hipMemcpyAsync(h_res, d_r, sizeof(gnsscorr_sdr_acq_result) * (size_t)n_rec * n_sv,
                       hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      gnsscorr_set_error("gnsscorr_sdr_acq_strong: %s", hipGetErrorString(e));
      rc = GNSSCORR_EDEVICE;
    }
  }
  cleanup();
  return rc;
}

extern "C" int gnsscorr_sdr_acq_sync(gnsscorr_sdr_acq_ctx* c) {
  if (!c) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" void* gnsscorr_sdr_acq_stream(gnsscorr_sdr_acq_ctx* c) {
  return c ? (void*)c->stream : nullptr;
}
