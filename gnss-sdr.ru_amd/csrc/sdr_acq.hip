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
//   sdr_strong_kernel  one workgroup per (record, sv, lcv), rows lcv2 = 0..3 in turn; row =
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
//
// Medium / weak acquisition (acquisition.cpp:309-570), same arithmetic:
//   sdr_prep_rows_kernel  doPrepIF at 1/10/310 ms into a per-record persistent
//                         row store (the object's baseband_rows member)
//   sdr_coh_kernel<WEAK>  one 1024-thread workgroup per (record, sv, row): ten
//                         1-ms inverse FFTs at once in LDS (80 KiB), the
//                         post-correlation DFT per delay column (v_dot2 =
//                         sse_cacc's pmaddwd), x86_cmag, and for weak the 15
//                         code-Doppler-shifted non-coherent sums in registers
//   sdr_select_mw_kernel  the strict-greater scan of doAcqMedium / doAcqWeak
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


typedef short short2_t __attribute__((ext_vector_type(2)));

// one radix-2 DIT butterfly of rank r with the reference's wrap points
// (fft.cpp:403-441: optional >>1 pre-scaling of both inputs, (b*w + 8192) >> 14
// in int32, int16 sum and difference), on packed {i, q} registers: A is the top
// element x[a], B the bottom x[a + 2^r].  w = {pack(wi, -wq), pack(wq, wi)}:
// the complex product's two components are v_dot2_i32_i16 with the rounding
// constant as the accumulator (exact: |b*w| <= 2^30 since |w| <= 2^14), and the
// int16 sum / difference are v_pk_add_u16 / v_pk_sub_u16 (wrapping, as the
// reference's int16 stores).
__device__ __forceinline__ void bfly(uint32_t& A, uint32_t& B, uint2 w, bool scale) {
  short2_t a = __builtin_bit_cast(short2_t, A), b = __builtin_bit_cast(short2_t, B);
  if (scale) { a = a >> (short)1; b = b >> (short)1; }
  // VOP3P v_dot2 with the rounding constant in an SGPR: the compiler's
  // v_dot2c form needs a v_mov into the accumulator per product.  volatile:
  // an inline asm has no implicit EXEC operand, and a non-volatile one may be
  // sunk or hoisted across the exec-mask writes of divergent branches
  // (track.hip's mad24 note); a volatile one stays where the source puts it.
  int32_t rnd, bi, bq;
  asm volatile("s_mov_b32 %0, 0x2000" : "=s"(rnd));
  asm volatile("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(bi) : "v"(b), "v"(w.x), "s"(rnd));
  asm volatile("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(bq) : "v"(b), "v"(w.y), "s"(rnd));
  bi >>= 14;
  bq >>= 14;
  const short2_t t = __builtin_bit_cast(short2_t, pack((int16_t)bi, (int16_t)bq));
  B = __builtin_bit_cast(uint32_t, a - t);
  A = __builtin_bit_cast(uint32_t, a + t);
}

// LDS twiddle entry for bfly from the packed (c, s) Q14 table
__device__ __forceinline__ uint2 tw_entry(uint32_t w) {
  const int16_t wi = lo16(w), wq = hi16(w);
  return make_uint2(pack(wi, (int16_t)-wq), pack(wq, wi));
}

// cmulsc(a, b, shift) with b given as tw_entry(b): the two products are
// v_dot2_i32_i16 with the rounding constant as the accumulator.  Exact when
// -b.q is an int16, i.e. b.q != -32768: the PRN spectra are within +-502
// (checked at context creation).
__device__ __forceinline__ uint32_t cmulsc_d2(uint32_t a, uint2 b2, int shift, bool sat) {
  const short2_t av = __builtin_bit_cast(short2_t, a);
  const int32_t rnd = 1 << (shift - 1);
  const int32_t ti = __builtin_amdgcn_sdot2(av, __builtin_bit_cast(short2_t, b2.x), rnd, false) >> shift;
  const int32_t tq = __builtin_amdgcn_sdot2(av, __builtin_bit_cast(short2_t, b2.y), rnd, false) >> shift;
  return sat ? pack(sat16(ti), sat16(tq)) : pack((int16_t)ti, (int16_t)tq);
}

// ---------------------------------------------------------------------------
// The reference's 11-rank radix-2 DIT (fft.cpp:156-180, rank/bfly loops
// :314-334) run as radix-8 passes in registers.  The butterflies of rank r
// pair positions a and a + 2^r and use twiddle (a mod 2^r) << (10 - r); the
// 2^R positions b + m*2^R0 (b with zero bits R0..R0+R-1) are closed under
// ranks R0..R0+R-1, so one thread can run those R ranks on them in registers
// with exactly the reference's butterflies and rounding.  11 ranks = passes
// at R0 = 0, 3, 6 (radix 8) and 9 (radix 4): four LDS round trips and
// barriers instead of eleven.
//   LDS layout: bit-reversed positions, padded by 8 words per 64 so that the
//   R0 = 3 pass (positions 64 apart) is bank-conflict free.
//   The R0 = 0 pass reads the natural-order input straight from global
//   memory: position 8g + m holds sample k = brev8(g) + 256 * brev3(m).
// ---------------------------------------------------------------------------
constexpr int kNP = kN + kN / 8;     // padded transform stride in LDS (words)
__device__ __forceinline__ int pad(int a) { return a + ((a >> 6) << 3); }
__device__ __forceinline__ int brev8(int g) { return (int)(__brev((uint32_t)g) >> 24); }
__device__ __forceinline__ int nat_k(int g, int m) {
  constexpr int kBrev3[8] = {0, 4, 2, 6, 1, 5, 3, 7};
  return brev8(g) + 256 * kBrev3[m];
}

// LDS twiddles: the 1024 entries of the reference table (tw_entry form), then
// per-pass copies for the R0 = 3 and R0 = 6 passes laid out [e][lo] (e = the
// group's twiddle slot, lo = b mod 2^R0).  Read from the main table, those two
// passes' lanes would hit one bank at power-of-two strides (8- to 16-way
// conflicts); from the [e][lo] copies consecutive lanes read consecutive
// entries.  The R0 = 0 pass reads broadcast entries, R0 = 9 stride 1 or 2.
constexpr int kTw3 = kN / 2;              // 7 x 8 entries
constexpr int kTw6 = kTw3 + 7 * 8;        // 7 x 64 entries
constexpr int kTwLds = kTw6 + 7 * 64;     // 1528 entries, 12 KiB

// the 2^R - 1 twiddles of one group: tws[2^s - 1 + i] for rank R0 + s, i < 2^s
template <int R0, int R, bool PT = false>
__device__ __forceinline__ void group_twiddles(uint2* tws, int lo, const uint2* tw) {
  if constexpr (PT && (R0 == 3 || R0 == 6)) {
    static_assert(R == 3, "per-pass tables are radix 8");
    const uint2* t = tw + (R0 == 3 ? kTw3 : kTw6);
#pragma unroll
    for (int e = 0; e < 7; e++) tws[e] = t[e * (1 << R0) + lo];
  } else {
#pragma unroll
    for (int s = 0; s < R; s++)
#pragma unroll
      for (int i = 0; i < (1 << s); i++)
        tws[(1 << s) - 1 + i] = tw[(lo + (i << R0)) << (kM - 1 - R0 - s)];
  }
}

// fill the LDS twiddles from the packed (c, s) Q14 table; T threads, caller
// syncs.  PT: also the per-pass copies.  They pay off only when a workgroup
// runs many transforms (sdr_coh_kernel: 10 per pass, 15 passes); for one
// transform per workgroup the extra staging costs more than the conflicts.
template <int T, bool PT>
__device__ __forceinline__ void stage_twiddles(uint2* tw, const uint32_t* __restrict__ glob) {
  for (int k = threadIdx.x; k < (PT ? kTwLds : kTw3); k += T) {
    int j = k;
    if (k >= kTw3) {
      const int r0 = k >= kTw6 ? 6 : 3, rel = k - (k >= kTw6 ? kTw6 : kTw3);
      const int e = rel >> r0, lo = rel & ((1 << r0) - 1);
      const int sl = e >= 3 ? 2 : (e >= 1 ? 1 : 0), i = e - ((1 << sl) - 1);
      j = (lo + (i << r0)) << (kM - 1 - r0 - sl);
    }
    tw[k] = tw_entry(glob[j]);
  }
}

// ranks R0 .. R0+R-1 on v[m] = x[b + m*2^R0]
template <int R0, int R, uint32_t MASK>
__device__ __forceinline__ void dit_group(uint32_t* v, const uint2* tws) {
#pragma unroll
  for (int s = 0; s < R; s++) {
    const bool scale = (MASK >> (R0 + s)) & 1u;
#pragma unroll
    for (int m = 0; m < (1 << R); m++)
      if (!(m & (1 << s))) bfly(v[m], v[m + (1 << s)], tws[(1 << s) - 1 + (m & ((1 << s) - 1))], scale);
  }
}

__device__ __forceinline__ void st_group8(uint32_t* x, int g, const uint32_t* v) {
  uint4* p = reinterpret_cast<uint4*>(x + pad(8 * g));
  p[0] = make_uint4(v[0], v[1], v[2], v[3]);
  p[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

// pass R0 = 0 on group g of one transform: in[m] = natural-order samples
// nat_k(g, m), already wiped off; result to LDS
template <uint32_t MASK>
__device__ __forceinline__ void dit_first(uint32_t* x, int g, uint32_t* v, const uint2* tw) {
  uint2 tws[7];
  group_twiddles<0, 3>(tws, 0, tw);
  dit_group<0, 3, MASK>(v, tws);
  st_group8(x, g, v);
}

// one in-LDS pass over F transforms (stride kNP) with T threads
template <int T, int F, int R0, int R, uint32_t MASK, bool PT = false>
__device__ __forceinline__ void dit_pass(uint32_t* x, const uint2* tw) {
  constexpr int E = 1 << R, G = kN >> R;
  static_assert(T % G == 0 || G % T == 0, "thread / group mapping");
  if constexpr (T % G == 0) {
    // fixed group per thread: twiddles loaded once, transforms f strided.
    // The empty asm keeps the per-group addresses and twiddles from being
    // hoisted out of an enclosing pass loop (they would stay live and spill).
    int g = threadIdx.x % G;
    asm volatile("" : "+v"(g));
    const int lo = g & ((1 << R0) - 1);
    const int b = lo | ((g >> R0) << (R0 + R));
    uint2 tws[E - 1];
    group_twiddles<R0, R, PT>(tws, lo, tw);
#pragma unroll 1
    for (int f = threadIdx.x / G; f < F; f += T / G) {
      uint32_t* xf = x + f * kNP;
      uint32_t v[E];
#pragma unroll
      for (int m = 0; m < E; m++) v[m] = xf[pad(b + (m << R0))];
      dit_group<R0, R, MASK>(v, tws);
#pragma unroll
      for (int m = 0; m < E; m++) xf[pad(b + (m << R0))] = v[m];
    }
  } else {
    for (int f = 0; f < F; f++)
#pragma unroll
      for (int u = 0; u < G / T; u++) {
        const int g = threadIdx.x + u * T, lo = g & ((1 << R0) - 1);
        const int b = lo | ((g >> R0) << (R0 + R));
        uint2 tws[E - 1];
        group_twiddles<R0, R, PT>(tws, lo, tw);
        uint32_t* xf = x + f * kNP;
        uint32_t v[E];
#pragma unroll
        for (int m = 0; m < E; m++) v[m] = xf[pad(b + (m << R0))];
        dit_group<R0, R, MASK>(v, tws);
#pragma unroll
        for (int m = 0; m < E; m++) xf[pad(b + (m << R0))] = v[m];
      }
  }
}

// the last pass (R0 = 9, radix 4) of a single transform into registers:
// v[m] = output position g + 512 m
template <uint32_t MASK>
__device__ __forceinline__ void dit_last_regs(const uint32_t* x, int g, uint32_t* v, const uint2* tw) {
  uint2 tws[3];
  group_twiddles<9, 2>(tws, g, tw);
#pragma unroll
  for (int m = 0; m < 4; m++) v[m] = x[pad(g + 512 * m)];
  dit_group<9, 2, MASK>(v, tws);
}

// whole transform of one row, T = 256 threads: first pass from the wiped-off
// natural-order samples produced by load(k), passes 3 and 6 in LDS; returns
// after the barrier that precedes the last pass
// load(k, m): the wiped-off natural-order sample k, the thread's m-th
template <uint32_t MASK, bool PT, class Load>
__device__ __forceinline__ void dit_row_256(uint32_t* x, const uint2* tw, Load load) {
  static_assert(kThreads == 256, "one radix-8 group per thread");
  const int g = threadIdx.x;
  uint32_t v[8];
#pragma unroll
  for (int m = 0; m < 8; m++) v[m] = load(nat_k(g, m), m);
  dit_first<MASK>(x, g, v, tw);
  __syncthreads();
  dit_pass<kThreads, 1, 3, 3, MASK, PT>(x, tw);
  __syncthreads();
  dit_pass<kThreads, 1, 6, 3, MASK, PT>(x, tw);
  __syncthreads();
}

__global__ __launch_bounds__(kThreads) void sdr_prep_kernel(
    const uint32_t* __restrict__ buff, const uint32_t* __restrict__ wipe,
    const uint32_t* __restrict__ tw_fwd, uint32_t* __restrict__ X, int saturate) {
  __shared__ uint32_t x[kNP];
  __shared__ uint2 tw[kTwLds];
  const int rec = blockIdx.x >> 2, j = blockIdx.x & 3;
  const uint32_t* src = buff + (size_t)rec * kN;
  const uint32_t* wp = wipe + (size_t)j * kN;
  stage_twiddles<kThreads, false>(tw, tw_fwd);
  __syncthreads();
  const bool sat = saturate != 0;
  dit_row_256<0u, false>(x, tw, [&](int k, int) { return cmulsc(src[k], wp[k], 14, sat); });   // R1: no scaling
  uint32_t* dst = X + ((size_t)rec * 4 + j) * kN;
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const int g = threadIdx.x + u * kThreads;
    uint32_t v[4];
    dit_last_regs<0u>(x, g, v, tw);
#pragma unroll
    for (int m = 0; m < 4; m++) dst[g + 512 * m] = v[m];
  }
}

// per-row result: (magnitude, index) of x86_cmag + x86_max
// One workgroup per (record, sv, lcv): the four 250-Hz sub-bins lcv2 of the
// 1-kHz shift run back to back, sharing the staged twiddles (with the per-pass
// copies) and the thread's eight PRN-spectrum samples.  Per-row result:
// (magnitude, index) of x86_cmag + x86_max at row_out[(rec, sv, row)], row =
// (lcv - lmin)*4 + lcv2.
__global__ __launch_bounds__(kThreads) void sdr_strong_kernel(
    const uint32_t* __restrict__ X, const uint32_t* __restrict__ codes,
    const uint32_t* __restrict__ tw_inv, const int32_t* __restrict__ svs, int n_sv, int lmin,
    int n_rows, int saturate, int2* __restrict__ row_out) {
  __shared__ uint32_t x[kNP];
  __shared__ uint2 tw[kTwLds];
  __shared__ int2 red[kThreads / 64];
  const int n_lcv = n_rows >> 2;
  const int l = blockIdx.x % n_lcv;
  const int s = (blockIdx.x / n_lcv) % n_sv;
  const int rec = blockIdx.x / (n_lcv * n_sv);
  const int lcv = lmin + l;
  const uint32_t* cr = codes + (size_t)svs[s] * kN;
  uint2 cv[8];   // the thread's PRN-spectrum samples in dot2 form
#pragma unroll
  for (int m = 0; m < 8; m++) cv[m] = tw_entry(cr[nat_k(threadIdx.x, m)]);
  stage_twiddles<kThreads, true>(tw, tw_inv);
  const bool sat = saturate != 0;
  for (int lcv2 = 0; lcv2 < 4; lcv2++) {
    __syncthreads();   // twiddles staged / the previous row's last pass has read x
    const uint32_t* xr = X + ((size_t)rec * 4 + lcv2) * kN;
    dit_row_256<kR2, true>(x, tw, [&](int k, int m) {
      return cmulsc_d2(xr[(k + lcv) & (kN - 1)], cv[m], 10, sat);
    });
    // last pass in registers, then x86_cmag (int32 wrap) + x86_max (first
    // index of the strict maximum, > 0): ties go to the smaller index
    int32_t best = 0, idx = 0;
#pragma unroll
    for (int u = 0; u < 2; u++) {
      const int g = threadIdx.x + u * kThreads;
      uint32_t v[4];
      dit_last_regs<kR2>(x, g, v, tw);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int32_t i = lo16(v[q]), qq = hi16(v[q]);
        const int32_t p = (int32_t)((uint32_t)(i * i) + (uint32_t)(qq * qq));
        if (p > best || (p == best && g + 512 * q < idx)) { best = p; idx = g + 512 * q; }
      }
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
      row_out[((size_t)rec * n_sv + s) * n_rows + l * 4 + lcv2] = r;
    }
  }
}

// The reference scans the rows in order with a strict '>' from 0, so it keeps
// the first row holding the maximum (if the maximum is > 0).  One wave per
// (record, sv): lane l scans rows l, l + 64, ... the same way, then the wave
// keeps the larger magnitude, and on equal magnitude the smaller row.
// Returns (magnitude, row) in every lane; magnitude 0 = no row beats 0.
__device__ __forceinline__ int2 first_max_row(const int2* __restrict__ rr, int n_rows, int lane) {
  int32_t mag = 0, row = 0x7fffffff;
  for (int r = lane; r < n_rows; r += 64) {
    const int32_t v = rr[r].x;
    if (v > mag) { mag = v; row = r; }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int32_t om = __shfl_xor(mag, o, 64), orow = __shfl_xor(row, o, 64);
    if (om > mag || (om == mag && orow < row)) { mag = om; row = orow; }
  }
  return make_int2(mag, row);
}

__global__ __launch_bounds__(64) void sdr_select_kernel(
    const int2* __restrict__ row_out, const int32_t* __restrict__ svs, int n_sv, int n_rec,
    int lmin, int n_rows, gnsscorr_sdr_acq_result* __restrict__ res) {
  const int g = blockIdx.x;   // (record, sv); doAcqStrong: lcv outer, lcv2 inner, strict >
  if (g >= n_rec * n_sv) return;
  const int2* rr = row_out + (size_t)g * n_rows;
  const int2 best = first_max_row(rr, n_rows, threadIdx.x);
  if (threadIdx.x != 0) return;
  gnsscorr_sdr_acq_result r = {};
  r.sv = svs[g % n_sv];
  if (best.x > 0) {
    const int row = best.y;
    r.code_phase = kN - rr[row].y;
    r.doppler = (lmin + (row >> 2)) * 1000 + (row & 3) * 250;
    r.magnitude = (uint32_t)best.x;
    r.row = row;
  }
  r.success = r.magnitude > 0u;   // THRESH_STRONG = 0 (config.h:72)
  res[g] = r;
}

// ---------------------------------------------------------------------------
// Medium / weak acquisition (acquisition.cpp:309-570)
// ---------------------------------------------------------------------------
constexpr int kStoreRows = 1240;      // baseband_rows (acquisition.cpp:107-110)
constexpr int kWipe = 10 * kN;        // 10-ms wipe-off tables, repeated (:123-137)
constexpr int kCoh = 1024;            // threads of the coherent kernels

__device__ __forceinline__ int32_t dot2(uint32_t a, uint32_t b, int32_t c) {
  // a.i*b.lo + a.q*b.hi + c in int32 (wrap): one pmaddwd half of sse_cacc
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, a), __builtin_bit_cast(short2_t, b),
                                c, false);
}

// doPrepIF for ms = 1, 10 or 310 ms (acquisition.cpp:191-236): one workgroup
// per (record, row r = j*ms + m): 1-ms block m mixed by the (-fif - 250 j)
// wipe-off at table offset (m % 10)*2048, forward FFT, stored as row r of the
// record's persistent row store.  Rows >= 4*ms are left as they are.
__global__ __launch_bounds__(kThreads) void sdr_prep_rows_kernel(
    const uint32_t* __restrict__ buff, int ms, const uint32_t* __restrict__ wipe10,
    const uint32_t* __restrict__ tw_fwd, uint32_t* __restrict__ store, int saturate) {
  __shared__ uint32_t x[kNP];
  __shared__ uint2 tw[kTwLds];
  const int nr = 4 * ms;
  const int rec = blockIdx.x / nr, r = blockIdx.x % nr, j = r / ms, m = r % ms;
  const uint32_t* src = buff + ((size_t)rec * ms + m) * kN;
  const uint32_t* wp = wipe10 + (size_t)j * kWipe + (size_t)(m % 10) * kN;
  stage_twiddles<kThreads, false>(tw, tw_fwd);
  __syncthreads();
  const bool sat = saturate != 0;
  dit_row_256<0u, false>(x, tw, [&](int k, int) { return cmulsc(src[k], wp[k], 14, sat); });
  uint32_t* dst = store + ((size_t)rec * kStoreRows + r) * kN;
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const int g = threadIdx.x + u * kThreads;
    uint32_t v[4];
    dit_last_regs<0u>(x, g, v, tw);
#pragma unroll
    for (int q = 0; q < 4; q++) dst[g + 512 * q] = v[q];
  }
}

__device__ __forceinline__ int weak_shift(int i, int lcv, int lcv2) {
#pragma clang fp contract(off)
  // acquisition.cpp:483-489: (double)i*.02*IF_SAMPLE_FREQUENCY*doppler/L1
  const double doppler = (double)(lcv * 1000) + (double)(float)(lcv2 * 250);
  const double cd = (double)i * .02 * 2048000.0 * doppler / 1.57542e9;
  return (int)floor(cd);
}

__device__ __forceinline__ void better(int32_t v, int32_t i, int32_t& best, int32_t& idx) {
  if (v > best || (v == best && i < idx)) { best = v; idx = i; }
}

// One workgroup per (record, sv, row).  Medium: row = (lcv - lmin)*4 + lcv2,
// one pass over store rows lcv2*20 + m (acquisition.cpp:338-345, the 20-row
// stride of the reference).  Weak: row = ((lcv - lmin)*4 + lcv2)*2 + k, 15
// passes i over rows lcv2*310 + i*20 + k*10 + m (:466-479).  A pass: the ten
// 1-ms rows read circularly from offset lcv, cmulsc by the PRN spectrum
// (shift 10 / 9), ten inverse FFTs at once in LDS (R2 scaling); then each
// delay column's post-correlation DFT against the 10 dft rows (sse_cacc as
// v_dot2 pairs, >> 16 to int16, :363-373) and x86_cmag.  Medium keeps the
// first strict maximum over the 10 x 2048 powers; weak adds the powers into
// per-thread int32 accumulators at column (c + shift) mod 2048 (:521-534),
// where a thread owns output columns tid and tid + 1024, and takes the
// maximum after the 15 passes.  Out: (max, flat index j*2048 + column).
template <bool WEAK>
__global__ __launch_bounds__(kCoh) void sdr_coh_kernel(
    const uint32_t* __restrict__ store, const uint32_t* __restrict__ codes,
    const uint32_t* __restrict__ tw_inv, const uint32_t* __restrict__ dft,
    const int32_t* __restrict__ svs, int n_sv, int lmin, int n_rows, int saturate,
    int2* __restrict__ row_out) {
  __shared__ uint32_t coh[10 * kNP];
  __shared__ uint2 tw[kTwLds];
  __shared__ int2 red[kCoh / 64];
  const int row = blockIdx.x % n_rows;
  const int s = (blockIdx.x / n_rows) % n_sv;
  const int rec = blockIdx.x / (n_rows * n_sv);
  const int lcv = lmin + (WEAK ? row >> 3 : row >> 2);
  const int lcv2 = WEAK ? (row >> 1) & 3 : row & 3;
  const int kk = WEAK ? row & 1 : 0;
  stage_twiddles<kCoh, true>(tw, tw_inv);
  const uint32_t* cr = codes + (size_t)svs[s] * kN;
  const uint32_t* rb = store + (size_t)rec * kStoreRows * kN;
  const bool sat = saturate != 0;
  // first radix-8 pass: thread t owns group g = t % 256 of the 1-ms rows
  // f = t / 256 + 4u (u < 3, f < 10); the eight PRN-spectrum samples it
  // multiplies are the same in every row and pass (re-read from L1/L2 rather
  // than held: the weak kernel is at the 128-VGPR limit of 1024 threads)
  const int g0 = threadIdx.x & 255, f0 = threadIdx.x >> 8;
  const int src0 = brev8(g0) + lcv;   // source column of sample k: (k + lcv) mod 2048
  __syncthreads();
  uint32_t acc[2][10];
#pragma unroll
  for (int q = 0; q < 2; q++)
#pragma unroll
    for (int j = 0; j < 10; j++) acc[q][j] = 0;
  int32_t best = 0, idx = 0;
  constexpr int kPasses = WEAK ? 15 : 1;
  for (int i = 0; i < kPasses; i++) {
    const int row0 = WEAK ? lcv2 * 310 + i * 20 + kk * 10 : lcv2 * 20;
#pragma unroll 1
    for (int u = 0; u < 3; u++) {
      int f = f0 + 4 * u;
      asm volatile("" : "+v"(f));   // per-pass addresses, not hoisted (see dit_pass)
      if (f < 10) {
        const uint32_t* rr = rb + (size_t)(row0 + f) * kN;
        uint32_t v[8];
#pragma unroll
        for (int m = 0; m < 8; m++)
          v[m] = cmulsc(rr[(nat_k(g0, m) - brev8(g0) + src0) & (kN - 1)], cr[nat_k(g0, m)], WEAK ? 9 : 10, sat);
        dit_first<kR2>(coh + f * kNP, g0, v, tw);
      }
    }
    __syncthreads();
    dit_pass<kCoh, 10, 3, 3, kR2, true>(coh, tw);
    __syncthreads();
    dit_pass<kCoh, 10, 6, 3, kR2, true>(coh, tw);
    __syncthreads();
    dit_pass<kCoh, 10, 9, 2, kR2>(coh, tw);
    __syncthreads();
    const int shift = WEAK ? weak_shift(i, lcv, lcv2) : 0;
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const int c_out = threadIdx.x + q * kCoh;
      const int c_in = (c_out - shift) & (kN - 1);
      uint32_t d[10];
#pragma unroll
      for (int m = 0; m < 10; m++) d[m] = coh[m * kNP + pad(c_in)];
#pragma unroll 2
      for (int j = 0; j < 10; j++) {
        int32_t ia = 0, qa = 0;
#pragma unroll
        for (int m = 0; m < 10; m++) {
          ia = dot2(d[m], dft[(j * 10 + m) * 2], ia);   // uniform: scalar loads
          qa = dot2(d[m], dft[(j * 10 + m) * 2 + 1], qa);
        }
        const int32_t ti = (int16_t)(ia >> 16), tq = (int16_t)(qa >> 16);
        const uint32_t p = (uint32_t)(ti * ti) + (uint32_t)(tq * tq);
        if (WEAK) acc[q][j] += p;
        else better((int32_t)p, j * kN + c_out, best, idx);
      }
    }
    if (WEAK) __syncthreads();   // coh is rewritten by the next pass
  }
  if (WEAK) {
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
      for (int j = 0; j < 10; j++) better((int32_t)acc[q][j], j * kN + threadIdx.x + q * kCoh, best, idx);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const int32_t ob = __shfl_xor(best, o, 64), oi = __shfl_xor(idx, o, 64);
    better(ob, oi, best, idx);
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = make_int2(best, idx);
  __syncthreads();
  if (threadIdx.x == 0) {
    int2 r = red[0];
    for (int w = 1; w < kCoh / 64; w++) {
      const int2 o = red[w];
      if (o.x > r.x || (o.x == r.x && o.y < r.y)) r = o;
    }
    if (r.x <= 0) r = make_int2(0, 0);
    row_out[blockIdx.x] = r;
  }
}

// per (record, sv): strict-greater scan over the rows in the reference's loop
// order (lcv, lcv2[, k]); code_phase = index % 2048 and doppler = lcv*1000 +
// lcv2*250 + (index / 2048)*25 (acquisition.cpp:397-405, :543-551)
__global__ __launch_bounds__(64) void sdr_select_mw_kernel(
    const int2* __restrict__ row_out, const int32_t* __restrict__ svs, int n_sv, int n_rec,
    int lmin, int n_rows, int weak, gnsscorr_sdr_acq_result* __restrict__ res) {
  const int g = blockIdx.x;   // (record, sv)
  if (g >= n_rec * n_sv) return;
  const int2* rr = row_out + (size_t)g * n_rows;
  const int2 best = first_max_row(rr, n_rows, threadIdx.x);
  if (threadIdx.x != 0) return;
  gnsscorr_sdr_acq_result r = {};
  r.sv = svs[g % n_sv];
  if (best.x > 0) {
    const int row = best.y, v = rr[row].y;
    const int lcv = lmin + (weak ? row >> 3 : row >> 2), lcv2 = weak ? (row >> 1) & 3 : row & 3;
    r.code_phase = v % kN;
    r.doppler = lcv * 1000 + lcv2 * 250 + (v / kN) * 25;
    r.magnitude = (uint32_t)best.x;
    r.row = row;
  }
  r.success = r.magnitude > 0u;   // THRESH_MEDIUM = THRESH_WEAK = 0 (config.h:73-74)
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
  // medium / weak: 10-ms wipe-offs, post-correlation DFT rows, and the
  // per-record persistent baseband_rows store (kStoreRows x 2048 CPX)
  uint32_t *d_wipe10 = nullptr, *d_dft = nullptr, *d_store = nullptr;
  size_t store_rec = 0;
};

extern "C" int gnsscorr_sdr_acq_destroy(gnsscorr_sdr_acq_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* ps[] = {c->d_wipe, c->d_codes, c->d_twf,    c->d_twi, c->d_X,    c->d_buff,
                c->d_svs,  c->d_rows,  c->d_res, c->d_wipe10, c->d_dft, c->d_store};
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
  uint32_t* w10 = (uint32_t*)malloc(sizeof(uint32_t) * (4 * (size_t)kWipe + 200));
  int rc = (h && tmp && w10) ? GNSSCORR_OK : GNSSCORR_ENOMEM;
  if (!rc) {
    // sine_gen over 10 ms (acquisition.cpp:123-128); the 1-ms tables are its head
    for (int j = 0; j < 4; j++) {
      gnsscorr_sdr_sine_gen((int16_t*)(w10 + (size_t)j * kWipe), -cfg->fif - 250.0 * j, 2048000.0,
                            kWipe);
      memcpy(h + (size_t)j * kN, w10 + (size_t)j * kWipe, sizeof(uint32_t) * kN);
    }
    gnsscorr_sdr_post_dft((int16_t*)(w10 + 4 * (size_t)kWipe));
    gnsscorr_sdr_prn_codes(tmp);
    memcpy(h + 4 * kN, tmp, sizeof(uint32_t) * 51 * kN);
    // cmulsc_d2 negates the code's Q component in int16 (sdr_strong_kernel):
    // -32768 would not be representable (the table is within +-502,
    // pinned by tests/test_codes_host.py)
    for (size_t k = 1; k < (size_t)51 * kN * 2; k += 2)
      if (((const int16_t*)tmp)[k] == -32768) {
        gnsscorr_set_error("gnsscorr_sdr_acq_create: PRN spectrum Q == -32768 is not "
                           "representable for the negated code product");
        rc = GNSSCORR_EINVAL;
        break;
      }
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
    if (e == hipSuccess) e = hipMalloc(&c->d_wipe10, sizeof(uint32_t) * 4 * kWipe);
    if (e == hipSuccess) e = hipMalloc(&c->d_dft, sizeof(uint32_t) * 200);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_wipe10, w10, sizeof(uint32_t) * 4 * kWipe, hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(c->d_dft, w10 + 4 * (size_t)kWipe, sizeof(uint32_t) * 200, hipMemcpyHostToDevice);
  }
  free(h);
  free(tmp);
  free(w10);
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
  hipLaunchKernelGGL(sdr_strong_kernel, dim3(n_rec * n_sv * (n_rows / 4)), dim3(kThreads), 0, c->stream,
                     c->d_X, c->d_codes, c->d_twi, d_svs, n_sv, lmin, n_rows, c->cfg.saturate,
                     c->d_rows);
  const int G = n_rec * n_sv;
  hipLaunchKernelGGL(sdr_select_kernel, dim3(G), dim3(64), 0, c->stream, c->d_rows,
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

// ============================================================================
// medium / weak acquisition (Acquisition::doPrepIF at 10 / 310 ms,
// doAcqMedium, doAcqWeak)
// ============================================================================
static int prep_ms(int type) {
  return type == GNSSCORR_SDR_ACQ_STRONG ? 1 : type == GNSSCORR_SDR_ACQ_MEDIUM ? 10
       : type == GNSSCORR_SDR_ACQ_WEAK   ? 310 : 0;
}

// the row store persists across calls (the Acquisition object's baseband_rows
// member); growing it keeps the rows of the records it already held and zeroes
// the new ones (the zero pages of the reference's fresh allocation)
static int ensure_store(gnsscorr_sdr_acq_ctx* c, int n_rec) {
  if ((size_t)n_rec <= c->store_rec) return GNSSCORR_OK;
  const size_t per = sizeof(uint32_t) * (size_t)kStoreRows * kN;
  uint32_t* p = nullptr;
  HIP_TRY(hipMalloc(&p, per * n_rec));
  hipError_t e = hipMemsetAsync((char*)p + per * c->store_rec, 0, per * (n_rec - c->store_rec),
                                c->stream);
  if (e == hipSuccess && c->store_rec)
    e = hipMemcpyAsync(p, c->d_store, per * c->store_rec, hipMemcpyDeviceToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    (void)hipFree(p);
    gnsscorr_set_error("gnsscorr_sdr_acq: row store: %s", hipGetErrorString(e));
    return GNSSCORR_EDEVICE;
  }
  (void)hipFree(c->d_store);
  c->d_store = p;
  c->store_rec = (size_t)n_rec;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_acq_prep_dev(gnsscorr_sdr_acq_ctx* c, int type, const int16_t* d_buff,
                                         int n_rec) {
  const int ms = prep_ms(type);
  if (!c || !d_buff || n_rec < 1 || ms == 0) {
    gnsscorr_set_error("gnsscorr_sdr_acq_prep_dev: bad arguments (type 0/1/2, n_rec >= 1)");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  int rc = ensure_store(c, n_rec);
  if (rc) return rc;
  hipLaunchKernelGGL(sdr_prep_rows_kernel, dim3(4 * ms * n_rec), dim3(kThreads), 0, c->stream,
                     (const uint32_t*)d_buff, ms, c->d_wipe10, c->d_twf, c->d_store,
                     c->cfg.saturate);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

static int mw_rows(int type, int doppmin, int doppmax, int* lmin, int* n_rows) {
  const int lo = doppmin / 1000, hi = doppmax / 1000;   // C truncation, as the reference
  if (type == GNSSCORR_SDR_ACQ_MEDIUM) {                // lcv <= doppmax/1000 (:324)
    if (hi < lo || lo < -kMaxLcv || hi > kMaxLcv) return GNSSCORR_EINVAL;
    *n_rows = 4 * (hi - lo + 1);
  } else if (type == GNSSCORR_SDR_ACQ_WEAK) {           // lcv < doppmax/1000 (:452)
    if (hi <= lo || lo < -kMaxLcv || hi > kMaxLcv + 1) return GNSSCORR_EINVAL;
    *n_rows = 8 * (hi - lo);
  } else {
    return GNSSCORR_EINVAL;
  }
  *lmin = lo;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_acq_search_dev(gnsscorr_sdr_acq_ctx* c, int type, int n_rec, int n_sv,
                                           const int32_t* d_svs, int doppmin, int doppmax,
                                           gnsscorr_sdr_acq_result* d_res) {
  if (!c || !d_svs || !d_res || n_rec < 1 || n_sv < 1) return GNSSCORR_EINVAL;
  int lmin = 0, n_rows = 0;
  if (mw_rows(type, doppmin, doppmax, &lmin, &n_rows)) {
    gnsscorr_set_error("gnsscorr_sdr_acq_search_dev: type must be MEDIUM (1) or WEAK (2) with "
                       "-100 <= doppmin/1000 <= doppmax/1000 <= 100 (weak: < and <= 101)");
    return GNSSCORR_EINVAL;
  }
  if ((size_t)n_rec > c->store_rec) {
    gnsscorr_set_error("gnsscorr_sdr_acq_search_dev: %d records but the row store holds %zu "
                       "(call gnsscorr_sdr_acq_prep_dev first)", n_rec, c->store_rec);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  int rc = grow((void**)&c->d_rows, &c->cap_rows, (size_t)n_rec * n_sv * n_rows, sizeof(int2));
  if (rc) return rc;
  const dim3 grid(n_rec * n_sv * n_rows);
  if (type == GNSSCORR_SDR_ACQ_WEAK)
    hipLaunchKernelGGL(sdr_coh_kernel<true>, grid, dim3(kCoh), 0, c->stream, c->d_store,
                       c->d_codes, c->d_twi, c->d_dft, d_svs, n_sv, lmin, n_rows,
                       c->cfg.saturate, c->d_rows);
  else
    hipLaunchKernelGGL(sdr_coh_kernel<false>, grid, dim3(kCoh), 0, c->stream, c->d_store,
                       c->d_codes, c->d_twi, c->d_dft, d_svs, n_sv, lmin, n_rows,
                       c->cfg.saturate, c->d_rows);
  const int G = n_rec * n_sv;
  hipLaunchKernelGGL(sdr_select_mw_kernel, dim3(G), dim3(64), 0, c->stream, c->d_rows,
                     d_svs, n_sv, n_rec, lmin, n_rows, type == GNSSCORR_SDR_ACQ_WEAK ? 1 : 0,
                     d_res);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_acq_acquire(gnsscorr_sdr_acq_ctx* c, int type, const int16_t* h_buff,
                                        int n_rec, int n_sv, const int32_t* h_svs, int doppmin,
                                        int doppmax, gnsscorr_sdr_acq_result* h_res) {
  if (!c || !h_buff || !h_svs || !h_res || n_rec < 1 || n_sv < 1) return GNSSCORR_EINVAL;
  if (type == GNSSCORR_SDR_ACQ_STRONG)
    return gnsscorr_sdr_acq_strong(c, h_buff, n_rec, n_sv, h_svs, doppmin, doppmax, h_res);
  int lmin = 0, n_rows = 0;
  if (mw_rows(type, doppmin, doppmax, &lmin, &n_rows)) {
    gnsscorr_set_error("gnsscorr_sdr_acq_acquire: bad type or Doppler range");
    return GNSSCORR_EINVAL;
  }
  for (int k = 0; k < n_sv; k++)
    if (h_svs[k] < 0 || h_svs[k] >= 32) {
      gnsscorr_set_error("gnsscorr_sdr_acq_acquire: sv %d out of range 0..31", h_svs[k]);
      return GNSSCORR_EINVAL;
    }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const int ms = prep_ms(type);
  size_t cap_b = 0, cap_s = 0, cap_r = 0;
  int16_t* d_b = nullptr;
  int32_t* d_s = nullptr;
  gnsscorr_sdr_acq_result* d_r = nullptr;
  auto cleanup = [&]() {
    (void)hipFree(d_b);
    (void)hipFree(d_s);
    (void)hipFree(d_r);
  };
  int rc;
  if ((rc = grow((void**)&d_b, &cap_b, (size_t)n_rec * ms * kN, sizeof(uint32_t))) ||
      (rc = grow((void**)&d_s, &cap_s, (size_t)n_sv, sizeof(int32_t))) ||
      (rc = grow((void**)&d_r, &cap_r, (size_t)n_rec * n_sv, sizeof(gnsscorr_sdr_acq_result)))) {
    cleanup();
    return rc;
  }
  hipError_t e = hipMemcpyAsync(d_b, h_buff, sizeof(uint32_t) * (size_t)n_rec * ms * kN,
                                hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_s, h_svs, sizeof(int32_t) * n_sv, hipMemcpyHostToDevice, c->stream);
  if (e != hipSuccess) {
    cleanup();
    gnsscorr_set_error("gnsscorr_sdr_acq_acquire: %s", hipGetErrorString(e));
    return GNSSCORR_EDEVICE;
  }
  rc = gnsscorr_sdr_acq_prep_dev(c, type, d_b, n_rec);
  if (!rc) rc = gnsscorr_sdr_acq_search_dev(c, type, n_rec, n_sv, d_s, doppmin, doppmax, d_r);
  if (!rc) {
    e = hipMemcpyAsync(h_res, d_r, sizeof(gnsscorr_sdr_acq_result) * (size_t)n_rec * n_sv,
                       hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
      gnsscorr_set_error("gnsscorr_sdr_acq_acquire: %s", hipGetErrorString(e));
      rc = GNSSCORR_EDEVICE;
    }
  } else {
    (void)hipStreamSynchronize(c->stream);
  }
  cleanup();
  return rc;
}
