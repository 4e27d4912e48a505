// acq.hip -- parallel code-phase acquisition on gfx950 (SoftGNSS semantics).
//
// Reference: POSTPROCESSING_SCILAB_RECEIVERS/GPS/L1/acquisition.sci:46-192
// (GLONASS: GLONASS/L1/acquisition.sci:46-198).  Per search group (PRN or
// FCH) and frequency bin:  X = fft(exp(i f 2 pi t) .* block),
// |ifft(X .* conj(fft(code)))|^2 for each 1-ms block, keep the block with the
// larger maximum, then peak / code phase / second peak outside +-1 chip.
//
// MI355X design
//  * N = samplesPerCode = 16368 = 16 * 3 * 11 * 31.  The four factors are
//    pairwise coprime, so the DFT is done as a Good-Thomas prime-factor FFT:
//    a 4-D DFT of shape 16 x 3 x 11 x 31 with NO inter-stage twiddles.  The
//    Ruritanian input map n(p) and CRT output map k(p) are pure index
//    permutations; they are folded into where data is read and written.
//  * One 1-ms row (16368 complex fp32 = 128 KiB) lives in LDS for the whole
//    transform; 528 work-items (9 wavefronts) each own one radix-16, one
//    3x11 or one radix-31 butterfly per pass: 3 LDS passes per transform.
//  * The IFFT is computed as a forward FFT of conj(Y) (|ifft(Y)| = |fft(conj Y)|/N),
//    so one kernel body serves both directions.
//  * Forward spectra of the wiped-off IF (shared by all codes) and of every
//    code replica are written to HBM already permuted into the correlation
//    kernel's LDS order (sigma = n^-1 o k), so the hot kernel streams both
//    operands with fully coalesced 8-byte loads and needs no gathers.
//  * The hot kernel fuses: conj(X)*F, 3 FFT passes, |.|^2, the per-row
//    max/argmax (first occurrence in natural order), the second peak outside
//    the +-spc window, and the best-of-blocks or non-coherent combine over
//    blocks -- the 16368-point power row never leaves registers.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "acq_ctx.h"
#include "if2.h"

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      gnsscorr_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                     \
      return GNSSCORR_EDEVICE;                                                          \
    }                                                                                   \
  } while (0)

// Diagnostic hook: tools/acq_stamps.hip defines ACQ_STAMP(i) to record
// s_memtime at phase boundaries; in the library it compiles to nothing.
// tools/acq_ablate.hip sets ACQ_SKIP to time the kernel with phases removed
// (1: no 3x11 pass, 2: no radix-31 pass, 4: no row statistics); 0 in the library.
#ifndef ACQ_SKIP
#define ACQ_SKIP 0
#endif
#ifndef ACQ_LOAD_AUX
#define ACQ_LOAD_AUX 0   // cache-policy bits of the X / F row loads
#endif
#ifndef ACQ_STAMP
#define ACQ_STAMP(i)
#endif
#ifndef ACQ_LDGROUP         // pipelined kernel: planes per group of row loads
#define ACQ_LDGROUP 16
#endif
#ifndef ACQ_PSTAMP          // pipelined kernel: (unit iteration, stamp id), tools/acq_pstamps.hip
#define ACQ_PSTAMP(it, i)
#endif

namespace {

constexpr int N = 16368;
constexpr int M16 = N / 16, M3 = N / 3, M11 = N / 11, M31 = N / 31;  // 1023 5456 1488 528
// CRT idempotents e_i = 1 mod N_i, 0 mod N_j (checked on the host at create)
constexpr int E16 = 15345, E3 = 10912, E11 = 5952, E31 = 528;
constexpr int kThreads = 512;           // 8 wavefronts -> up to 256 VGPRs each
// Spectra rows in HBM are padded to 16 planes x 1024 complex (128 KiB) so the
// radix-16 loads are 16-byte aligned: LDS position a*1023+g <-> a*1024+g.
#ifndef ACQ_PLANE
#define ACQ_PLANE 1024
#endif
constexpr int kPlane = ACQ_PLANE;
constexpr int NPAD = 16 * kPlane;
constexpr int kGroups31 = N / 31;       // 528 radix-31 groups
constexpr int kLeft = kGroups31 - kThreads;  // 16 groups done as direct dot products

constexpr float kCos11[11] = {1.000000000e+00f, 8.412535328e-01f, 4.154150130e-01f, -1.423148383e-01f, -6.548607339e-01f, -9.594929736e-01f, -9.594929736e-01f, -6.548607339e-01f, -1.423148383e-01f, 4.154150130e-01f, 8.412535328e-01f};
constexpr float kSin11[11] = {0.000000000e+00f, 5.406408175e-01f, 9.096319954e-01f, 9.898214419e-01f, 7.557495744e-01f, 2.817325568e-01f, -2.817325568e-01f, -7.557495744e-01f, -9.898214419e-01f, -9.096319954e-01f, -5.406408175e-01f};
constexpr float kCos31[31] = {1.000000000e+00f, 9.795299413e-01f, 9.189578116e-01f, 8.207634412e-01f, 6.889669191e-01f, 5.289640103e-01f, 3.473052528e-01f, 1.514277775e-01f, -5.064916884e-02f, -2.506525323e-01f, -4.403941516e-01f, -6.121059825e-01f, -7.587581227e-01f, -8.743466161e-01f, -9.541392564e-01f, -9.948693234e-01f, -9.948693234e-01f, -9.541392564e-01f, -8.743466161e-01f, -7.587581227e-01f, -6.121059825e-01f, -4.403941516e-01f, -2.506525323e-01f, -5.064916884e-02f, 1.514277775e-01f, 3.473052528e-01f, 5.289640103e-01f, 6.889669191e-01f, 8.207634412e-01f, 9.189578116e-01f, 9.795299413e-01f};
constexpr float kSin31[31] = {0.000000000e+00f, 2.012985201e-01f, 3.943558551e-01f, 5.712682151e-01f, 7.247927872e-01f, 8.486442575e-01f, 9.377521321e-01f, 9.884683243e-01f, 9.987165072e-01f, 9.680771189e-01f, 8.978045396e-01f, 7.907757369e-01f, 6.513724827e-01f, 4.853019625e-01f, 2.993631230e-01f, 1.011683220e-01f, -1.011683220e-01f, -2.993631230e-01f, -4.853019625e-01f, -6.513724827e-01f, -7.907757369e-01f, -8.978045396e-01f, -9.680771189e-01f, -9.987165072e-01f, -9.884683243e-01f, -9.377521321e-01f, -8.486442575e-01f, -7.247927872e-01f, -5.712682151e-01f, -3.943558551e-01f, -2.012985201e-01f};
constexpr float kCos16[16] = {1.0f, 9.238795325e-01f, 7.071067812e-01f, 3.826834324e-01f, 0.0f, -3.826834324e-01f, -7.071067812e-01f, -9.238795325e-01f, -1.0f, -9.238795325e-01f, -7.071067812e-01f, -3.826834324e-01f, 0.0f, 3.826834324e-01f, 7.071067812e-01f, 9.238795325e-01f};
constexpr float kSin16[16] = {0.0f, 3.826834324e-01f, 7.071067812e-01f, 9.238795325e-01f, 1.0f, 9.238795325e-01f, 7.071067812e-01f, 3.826834324e-01f, 0.0f, -3.826834324e-01f, -7.071067812e-01f, -9.238795325e-01f, -1.0f, -9.238795325e-01f, -7.071067812e-01f, -3.826834324e-01f};
constexpr float kSqrt3_2 = 8.660254038e-01f;

// Complex values live in packed fp32 pairs (v2f): gfx950 executes v_pk_fma_f32 /
// v_pk_add_f32 on both halves in one instruction, and re/im swaps and sign
// flips fold into the op_sel / neg modifiers, so the DFTs below are written
// with explicit swaps instead of scalar re/im arithmetic.
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f swp(v2f v) { return __builtin_shufflevector(v, v, 1, 0); }
__device__ __forceinline__ v2f bc(float c) { return (v2f){c, c}; }
// -i v = (v.y, -v.x)
__device__ __forceinline__ v2f mul_mi(v2f v) { return swp(v) * (v2f){1.f, -1.f}; }
// v * (c + i s) for constants c, s
__device__ __forceinline__ v2f cmulc(v2f v, float c, float s) {
  return v * bc(c) + swp(v) * (v2f){-s, s};
}
__device__ __forceinline__ v2f ld2(const float2& f) { return (v2f){f.x, f.y}; }
__device__ __forceinline__ float2 st2(v2f v) { return make_float2(v.x, v.y); }

// ---- small forward DFTs (W = exp(-2 pi i / P)) --------------------------------
__device__ __forceinline__ void dft4(v2f& a, v2f& b, v2f& c, v2f& d) {
  const v2f t0 = a + c, t1 = a - c, t2 = b + d, t3 = b - d;
  a = t0 + t2;
  c = t0 - t2;
  const v2f s3 = swp(t3);
  b = __builtin_elementwise_fma(s3, (v2f){1.f, -1.f}, t1);   // t1 - i t3
  d = __builtin_elementwise_fma(s3, (v2f){-1.f, 1.f}, t1);   // t1 + i t3
}

// In place: on return x[k] = X[k].
__device__ __forceinline__ void dft16(v2f (&x)[16]) {
#pragma unroll
  for (int n2 = 0; n2 < 4; n2++) dft4(x[n2], x[4 + n2], x[8 + n2], x[12 + n2]);
#pragma unroll
  for (int k1 = 1; k1 < 4; k1++)
#pragma unroll
    for (int n2 = 1; n2 < 4; n2++) {
      const int m = n2 * k1;
      x[4 * k1 + n2] = cmulc(x[4 * k1 + n2], kCos16[m], -kSin16[m]);
    }
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++) dft4(x[4 * k1], x[4 * k1 + 1], x[4 * k1 + 2], x[4 * k1 + 3]);
  // X[k1 + 4 k2] sits in slot 4 k1 + k2: transpose the 4x4 block (register renaming)
  v2f y[16];
#pragma unroll
  for (int i = 0; i < 16; i++) y[i] = x[i];
#pragma unroll
  for (int k1 = 0; k1 < 4; k1++)
#pragma unroll
    for (int k2 = 0; k2 < 4; k2++) x[k1 + 4 * k2] = y[4 * k1 + k2];
}

__device__ __forceinline__ void dft3(v2f& x0, v2f& x1, v2f& x2) {
  const v2f s = x1 + x2, d = x1 - x2;
  const v2f t = x0 - bc(0.5f) * s;
  x0 = x0 + s;
  const v2f sd = swp(d);   // -/+ i sqrt(3)/2 (x1 - x2)
  x1 = __builtin_elementwise_fma(sd, (v2f){kSqrt3_2, -kSqrt3_2}, t);
  x2 = __builtin_elementwise_fma(sd, (v2f){-kSqrt3_2, kSqrt3_2}, t);
}

template <int P>
__device__ __forceinline__ float ctab(int k) { return P == 11 ? kCos11[k] : kCos31[k]; }
template <int P>
__device__ __forceinline__ float stab(int k) { return P == 11 ? kSin11[k] : kSin31[k]; }

// Symmetric prime-length DFT: X_m = A_m - i B_m, X_{P-m} = A_m + i B_m with
// A_m = x0 + sum_j cos(2 pi jm/P)(x_j + x_{P-j}), B_m = sum_j sin(..)(x_j - x_{P-j}).
template <int P>
__device__ __forceinline__ void dftp(v2f (&x)[P]) {
  constexpr int H = (P - 1) / 2;
  v2f s[H + 1], d[H + 1];
#pragma unroll
  for (int j = 1; j <= H; j++) {
    s[j] = x[j] + x[P - j];
    d[j] = x[j] - x[P - j];
  }
  const v2f x0 = x[0];
  v2f X0 = x0;
#pragma unroll
  for (int j = 1; j <= H; j++) X0 += s[j];
  x[0] = X0;
#pragma unroll
  for (int m = 1; m <= H; m++) {
    v2f A = x0, B = (v2f){0.f, 0.f};
#pragma unroll
    for (int j = 1; j <= H; j++) {
      const int q = (j * m) % P;
      A += bc(ctab<P>(q)) * s[j];
      B += bc(stab<P>(q)) * d[j];
    }
    const v2f sb = swp(B);
    x[m] = __builtin_elementwise_fma(sb, (v2f){1.f, -1.f}, A);        // A - i B
    x[P - m] = __builtin_elementwise_fma(sb, (v2f){-1.f, 1.f}, A);    // A + i B
  }
}

// ---- index maps --------------------------------------------------------------
// LDS position p = a*1023 + (b*11 + c)*31 + d
__device__ __forceinline__ int in_index(int p) {  // Ruritanian input map n(p)
  const int d = p % 31, c = (p / 31) % 11, b = (p / 341) % 3, a = p / 1023;
  int n = a * M16 + b * M3 + c * M11 + d * M31;
  n %= N;
  return n;
}

// ---- the three in-LDS passes (16, 3x11, 31) ----------------------------------
// Correlation-kernel first pass straight from HBM/L2: every thread owns the
// two adjacent radix-16 groups g = 2t, 2t+1 and reads them as ONE 16-byte
// buffer load per plane a (scalar plane offset a*8 KiB, 32-bit lane offset),
// forms D = conj(X) * F, runs both DFT16s in registers and writes LDS once.
typedef float f4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));

// Frequency bins on the fs/N grid share one spectrum: X_f[k] = X_f0[k - m]
// for f = f0 + m*fs/N (exact circular shift).  In prime-factor coordinates a
// shift by m subtracts (15m mod 16, 2m mod 3, 4m mod 11, m mod 31) from the
// (a, b, c, d) of every position, so the X read below is still one plane per
// a and an (almost always) contiguous pair of groups.
struct Shift { int a, b, c, d; };

__device__ __forceinline__ int shift_group(int g, const Shift& s) {
  const int d = g % 31, bc = g / 31, c = bc % 11, b = bc / 11;
  int b2 = b - s.b, c2 = c - s.c, d2 = d - s.d;
  b2 += b2 < 0 ? 3 : 0;
  c2 += c2 < 0 ? 11 : 0;
  d2 += d2 < 0 ? 31 : 0;
  return (b2 * 11 + c2) * 31 + d2;
}

__device__ __forceinline__ void load_mul_pass16(const float2* __restrict__ Xb,
                                                const float2* __restrict__ Fc, float2* lds,
                                                int t, const Shift& sh) {
  const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)Xb, 0, NPAD * 8, 0x00020000);
  const auto rf = __builtin_amdgcn_make_buffer_rsrc((void*)Fc, 0, NPAD * 8, 0x00020000);
  const int g0 = 2 * t;
  const int voff = g0 * 8;
  v2f x0[16], x1[16];
  if (sh.a == 0 && sh.b == 0 && sh.c == 0 && sh.d == 0) {   // uniform branch
#pragma unroll
    for (int a = 0; a < 16; a++) {
      const f4v u = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, voff, a * kPlane * 8, ACQ_LOAD_AUX));
      const f4v f = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rf, voff, a * kPlane * 8, ACQ_LOAD_AUX));
      // conj(u) * f = u.re * f + u.im * (f.im, -f.re)
      const v2f f0 = (v2f){f.x, f.y}, f1 = (v2f){f.z, f.w};
      x0[a] = bc(u.x) * f0 + bc(u.y) * mul_mi(f0);
      x1[a] = bc(u.z) * f1 + bc(u.w) * mul_mi(f1);
    }
  } else {
    const int v0 = shift_group(g0 < M16 ? g0 : 0, sh) * 8;
    const int v1 = shift_group(g0 + 1 < M16 ? g0 + 1 : 0, sh) * 8;
#pragma unroll
    for (int a = 0; a < 16; a++) {
      const int pa = ((a - sh.a) & 15) * kPlane * 8;
      const f2v u0 = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rx, v0, pa, ACQ_LOAD_AUX));
      const f2v u1 = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rx, v1, pa, ACQ_LOAD_AUX));
      const f4v f = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rf, voff, a * kPlane * 8, ACQ_LOAD_AUX));
      const v2f f0 = (v2f){f.x, f.y}, f1 = (v2f){f.z, f.w};
      x0[a] = bc(u0.x) * f0 + bc(u0.y) * mul_mi(f0);
      x1[a] = bc(u1.x) * f1 + bc(u1.y) * mul_mi(f1);
    }
  }
  dft16(x0);
  dft16(x1);
  const bool two = g0 + 1 < M16;
#pragma unroll
  for (int a = 0; a < 16; a++) {
    lds[a * M16 + g0] = st2(x0[a]);
    if (two) lds[a * M16 + g0 + 1] = st2(x1[a]);
  }
}

__device__ __forceinline__ void pass33(float2* lds, int t) {
  if (t >= 16 * 31) return;
  const int a = t / 31, d = t % 31;
  float2* base = lds + a * M16 + d;
  v2f v[3][11];
#pragma unroll
  for (int b = 0; b < 3; b++)
#pragma unroll
    for (int c = 0; c < 11; c++) v[b][c] = ld2(base[(b * 11 + c) * 31]);
#pragma unroll
  for (int c = 0; c < 11; c++) dft3(v[0][c], v[1][c], v[2][c]);
#pragma unroll
  for (int b = 0; b < 3; b++) dftp<11>(v[b]);
#pragma unroll
  for (int b = 0; b < 3; b++)
#pragma unroll
    for (int c = 0; c < 11; c++) base[(b * 11 + c) * 31] = st2(v[b][c]);
}

// dim-31 pass, leftover groups 512..527: thread t < 496 computes output m of
// group 512 + t/31 as a direct 31-term DFT sum (twiddles from an LDS table).
__device__ __forceinline__ float2 dft31_single(const float2* lds, const float2* tw, int t) {
  const int grp = kThreads + t / 31, m = t % 31;
  const float2* x = lds + grp * 31;
  float re = 0.f, im = 0.f;
  int q = 0;
#pragma unroll
  for (int j = 0; j < 31; j++) {
    const float2 v = x[j], w = tw[q];  // w = exp(-2 pi i q / 31)
    re = fmaf(v.x, w.x, fmaf(-v.y, w.y, re));
    im = fmaf(v.x, w.y, fmaf(v.y, w.x, im));
    q += m;
    if (q >= 31) q -= 31;
  }
  return make_float2(re, im);
}

__device__ __forceinline__ void init_tw31(float2* tw) {
  if (threadIdx.x < 31) tw[threadIdx.x] = make_float2(kCos31[threadIdx.x], -kSin31[threadIdx.x]);
}

// natural output index of LDS position t*31 + d': k = (a E16 + b E3 + c E11 + d' E31) mod N
__device__ __forceinline__ int out_base(int t) {
  const int a = t / 33, bc = t % 33, b = bc / 11, c = bc % 11;
  return (a * E16 + b * E3 + c * E11) % N;  // < 2^31: 32-bit modulo
}

// ---- forward spectra: wiped-off IF rows and code rows --------------------------
// The forward transforms are latency-bound (82 rows for a GPS search), so each
// row is split over many small workgroups with the prime-factor structure:
//   K1: wipe-off + radix-16 pass, 4 workgroups x 256 groups per row -> HBM
//       staging T[row][a'][1024]
//   K2: the 16 independent 1023-point (3 x 11 x 31) sub-transforms of a row,
//       one wavefront each, written straight to the correlation layout (sigma).
// mode 0: IF row = (freq_id, block); x[n] = IF[block][n] * exp(i f ((n*2)*pi)*ts)
//         with coh > 1 a block is coh code periods and x[n] = sum over p < coh of
//         the wiped-off sample n + p*N (phase index n + p*N): the coh*N-point
//         spectrum of acquisition.sci's settings.acqCohIntegration-ms blocks
//         against repmat(code, coh) is nonzero only at multiples of coh, where it
//         equals this folded N-point spectrum times coh x the 1-ms code spectrum,
//         and its inverse is the same N-periodic power row (GLONASS
//         acquisition.sci:52-72, 113-135: "The rest are copies of the first 1msec")
// mode 1: code row c; x[n] = code[c][n]
__device__ __forceinline__ double grid_residue(double f, double delta) {
  double r = fmod(f, delta);
  return r < 0 ? r + delta : r;
}

constexpr int kFuseClass = 64;   // frequency tables this short are classified inside fwd16
constexpr int kFwd1Threads = 256;
constexpr int kFwd1G = kFwd1Threads / 16;   // radix-16 columns g per workgroup
// One workgroup = 16 columns g of one row: every thread makes ONE input sample
// (a, g) -- the wipe-off's fp64 sincos spread over 64 workgroups per row, not
// 16 per thread -- then 16 threads run the radix-16 of their column.
__global__ __launch_bounds__(kFwd1Threads) void acq_fwd16_kernel(
    const int8_t* __restrict__ src, int iq, int n_blocks, const double* __restrict__ freqs,
    double ts, int mode, float2* __restrict__ stage, const double* __restrict__ cfreqs,
    const int* __restrict__ n_rows_dev, int coh, int n_rows, int fuse_n, double delta,
    int4* __restrict__ fmap_out, double* __restrict__ cfreq_out, int* __restrict__ nclass_out) {
  __shared__ float2 xs[kFwd1G][17];
  __shared__ double s_r[kFuseClass], s_cf[kFuseClass];
  __shared__ int s_l[kFuseClass], s_nc;
  const int chunks = (M16 + kFwd1G - 1) / kFwd1G;
  int n_cls_rows = n_rows_dev ? -1 : n_rows;
  if (fuse_n > 0) {
    // acq_classify_kernel folded in for short frequency tables: every workgroup
    // classifies the table in LDS (fuse_n <= kFuseClass lanes), workgroup 0
    // publishes the map for the later kernels
    const int t = threadIdx.x;
    if (t < fuse_n) s_r[t] = grid_residue(freqs[t], delta);
    __syncthreads();
    if (t < fuse_n) {
      int l = t;
      for (int j = 0; j < t; j++)
        if (s_r[j] == s_r[t]) { l = j; break; }
      s_l[t] = l;
    }
    __syncthreads();
    if (t < fuse_n) {
      const int l = s_l[t];
      int cls = 0;
      for (int k = 0; k < l; k++) cls += s_l[k] == k;
      if (l == t) s_cf[cls] = s_r[t];
      if (blockIdx.x == 0) {
        const double q = rint((freqs[t] - s_r[t]) / delta);
        int mN = (fabs(q) < 1e8 ? (int)q : 0) % N;
        mN += mN < 0 ? N : 0;
        fmap_out[t] = make_int4(cls, (15 * mN) & 15, (2 * mN) % 3, ((4 * mN) % 11) * 32 + mN % 31);
        if (l == t) cfreq_out[cls] = s_r[t];
      }
    }
    if (t == 0) {
      int cnt = 0;
      for (int k = 0; k < fuse_n; k++) cnt += s_l[k] == k;
      s_nc = cnt;
      if (blockIdx.x == 0) *nclass_out = cnt;
    }
    __syncthreads();
    n_cls_rows = s_nc * n_blocks;
    cfreqs = s_cf;
  } else if (n_rows_dev) {
    n_cls_rows = *n_rows_dev * n_blocks;
  }
  // grid-stride over (row, chunk): only the spectrum-class rows exist
  const int total = n_cls_rows * chunks;
  for (int w = blockIdx.x; w < total; w += gridDim.x) {
  const int row = w / chunks, g0 = (w % chunks) * kFwd1G;
  const int a = threadIdx.x >> 4, gl = threadIdx.x & 15, g = g0 + gl;
  if (g < M16) {
    const int n0 = in_index(a * M16 + g);
    float2 v;
    if (mode == 0) {
      const int cls = row / n_blocks, blk = row % n_blocks;
      const double f = cfreqs[cls];
      const bool cplx = iq & GNSSCORR_IF_IQ, pk = iq & GNSSCORR_IF_PACKED2;
      const int ne = cplx ? 2 : 1;
      const long e0 = (long)blk * coh * N * ne;   // first element of the block
      double re = 0.0, im = 0.0;
      for (int p = 0; p < coh; p++) {
        const int n = n0 + p * N;
        const double I = (double)if_elem(src, e0 + (long)ne * n, pk);
        const double Q = cplx ? (double)if_elem(src, e0 + 2L * n + 1, pk) : 0.0;
        // acquisition.sci:61-62, 107: phasePoints = (0:coh*N-1)*2*%pi*ts; exp(i f pp)
        const double th = f * ((((double)n * 2.0) * M_PI) * ts);
        double sn, cs;
        sincos(th, &sn, &cs);
        re += I * cs - Q * sn;
        im += I * sn + Q * cs;
      }
      v = make_float2((float)re, (float)im);
    } else {
      v = make_float2((float)src[(long)row * N + n0], 0.f);
    }
    xs[gl][a] = v;
  }
  __syncthreads();
  if (threadIdx.x < kFwd1G && g0 + threadIdx.x < M16) {
    const int gg = g0 + threadIdx.x;
    v2f x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = ld2(xs[threadIdx.x][k]);
    dft16(x);
    float2* o = stage + (long)row * NPAD + gg;
#pragma unroll
    for (int k = 0; k < 16; k++) o[k * kPlane] = st2(x[k]);
  }
  __syncthreads();   // xs is rewritten by the next item
  }
}

// The 1023-point (3 x 11 x 31) sub-transform of plane a of a row, 512 threads:
// dft3 over b for the 341 (c, d) columns, dft11 over c for the 93 (b, d)
// columns, then the 33 radix-31 groups split into their 16 output pairs
// (X_0 and X_m / X_{31-m} of the symmetric form): 528 tasks, one round.  The
// scatter targets (sigma) are fetched before the first barrier.
constexpr int kFwd2Threads = 512;
__global__ __launch_bounds__(kFwd2Threads) void acq_fwd1023_kernel(
    const float2* __restrict__ stage, const int* __restrict__ sigma, float2* __restrict__ out,
    int n_blocks, const int* __restrict__ n_rows_dev, int n_rows) {
  __shared__ float2 sub[M16 + 1];
  const int total = (n_rows_dev ? *n_rows_dev * n_blocks : n_rows) * 16;
  const int t = threadIdx.x;
  for (int w = blockIdx.x; w < total; w += gridDim.x) {
    const int row = w >> 4, a = w & 15;
    // radix-31 tasks of this thread: k = t and t + 512 (k < 528)
    int dst0[2], dst1[2];
#pragma unroll
    for (int r = 0; r < 2; r++) {
      const int k = t + r * kFwd2Threads;
      dst0[r] = dst1[r] = 0;
      if (k < 33 * 16) {
        const int grp = k >> 4, m = k & 15, p0 = a * M16 + grp * 31;
        dst0[r] = sigma[p0 + m];
        dst1[r] = m ? sigma[p0 + 31 - m] : 0;
      }
    }
    const float2* in = stage + (long)row * NPAD + a * kPlane;
    for (int i = t; i < M16; i += kFwd2Threads) sub[i] = in[i];
    __syncthreads();
    if (t < 11 * 31) {   // radix 3 over b, column (c, d)
      const int c = t / 31, d = t % 31;
      v2f x0 = ld2(sub[c * 31 + d]), x1 = ld2(sub[(11 + c) * 31 + d]),
          x2 = ld2(sub[(22 + c) * 31 + d]);
      dft3(x0, x1, x2);
      sub[c * 31 + d] = st2(x0);
      sub[(11 + c) * 31 + d] = st2(x1);
      sub[(22 + c) * 31 + d] = st2(x2);
    }
    __syncthreads();
    if (t < 3 * 31) {    // radix 11 over c, column (b, d)
      const int b = t / 31, d = t % 31;
      v2f v[11];
#pragma unroll
      for (int c = 0; c < 11; c++) v[c] = ld2(sub[(b * 11 + c) * 31 + d]);
      dftp<11>(v);
#pragma unroll
      for (int c = 0; c < 11; c++) sub[(b * 11 + c) * 31 + d] = st2(v[c]);
    }
    __syncthreads();
    float2* o = out + (long)row * NPAD;
#pragma unroll
    for (int r = 0; r < 2; r++) {   // radix 31: (group, output pair m)
      const int k = t + r * kFwd2Threads;
      if (k >= 33 * 16) break;
      const int grp = k >> 4, m = k & 15;
      const float2* x = &sub[grp * 31];
      const v2f x0 = ld2(x[0]);
      if (m == 0) {
        v2f X0 = x0;
#pragma unroll
        for (int j = 1; j <= 15; j++) X0 += ld2(x[j]) + ld2(x[31 - j]);
        o[dst0[r]] = st2(X0);
      } else {
        v2f A = x0, B = (v2f){0.f, 0.f};
        int q = m;
#pragma unroll
        for (int j = 1; j <= 15; j++) {   // q = j*m mod 31
          const v2f xj = ld2(x[j]), xn = ld2(x[31 - j]);
          A += bc(kCos31[q]) * (xj + xn);
          B += bc(kSin31[q]) * (xj - xn);
          q += m;
          if (q >= 31) q -= 31;
        }
        const v2f sb = swp(B);
        o[dst0[r]] = st2(__builtin_elementwise_fma(sb, (v2f){1.f, -1.f}, A));   // A - i B
        o[dst1[r]] = st2(__builtin_elementwise_fma(sb, (v2f){-1.f, 1.f}, A));   // A + i B
      }
    }
    __syncthreads();   // sub is reloaded by the next item
  }
}

// Spectrum classes: frequencies with the same residue r = f mod fs/N share one
// forward spectrum, computed AT r; bin f = r + m*fs/N reads it circularly
// shifted by m (exact identity: exp(i 2 pi m n / N) modulation).  The class
// spectrum depends on r alone, so results do not depend on which other
// frequencies are in the list (sharding / ordering invariant).
// fmap[i] = {class, 15m mod 16, 2m mod 3, (4m mod 11) * 32 + m mod 31};
// cfreq[class] = r.

constexpr int kClassLds = 2048;   // frequencies classified in LDS (larger tables: global scratch)
__global__ __launch_bounds__(1024) void acq_classify_kernel(const double* __restrict__ freqs,
                                                            int n, double delta,
                                                            int4* __restrict__ fmap,
                                                            double* __restrict__ cfreq,
                                                            int* __restrict__ n_classes,
                                                            double* __restrict__ resid) {
  extern __shared__ double s_cls[];   // [n] residues, then [n] int4 (n <= kClassLds)
  const bool lds = n <= kClassLds;
  double* R = lds ? s_cls : resid;
  int4* F = lds ? reinterpret_cast<int4*>(s_cls + ((n + 1) & ~1)) : fmap;
  // pass 0: every residue once (fmod is a long fp64 sequence)
  for (int i = threadIdx.x; i < n; i += blockDim.x) R[i] = grid_residue(freqs[i], delta);
  __syncthreads();
  // pass 1: leader = first j with the same residue; shift m = (f - r) / delta
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double f = freqs[i], r = R[i];
    int l = i;
    for (int j = 0; j < i; j++)
      if (R[j] == r) { l = j; break; }
    const double q = rint((f - r) / delta);
    F[i] = make_int4(l, fabs(q) < 1e8 ? (int)q : 0, 0, 0);
  }
  __syncthreads();
  // pass 2: class id = number of leaders before the leader
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int4 v = F[i];
    int cls = 0;
    for (int k = 0; k < v.x; k++) cls += F[k].x == k;
    int mN = v.y % N;
    mN += mN < 0 ? N : 0;
    F[i].z = cls;
    F[i].w = mN;
  }
  // class count: every thread counts its own entries (one thread walking the
  // table was a dependent LDS/global load per entry)
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  int mine = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) mine += F[i].x == i;
  atomicAdd(&s_cnt, mine);
  __syncthreads();
  if (threadIdx.x == 0) *n_classes = s_cnt;
  // pass 3: class frequencies and the packed shift coordinates
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int4 v = F[i];
    if (v.x == i) cfreq[v.z] = R[i];
    const int mN = v.w;
    fmap[i] = make_int4(v.z, (15 * mN) & 15, (2 * mN) % 3, ((4 * mN) % 11) * 32 + mN % 31);
  }
}

// ---- block-level reductions ---------------------------------------------------
struct PeakSlot {
  float v;
  int k;
};

__device__ __forceinline__ bool better(float v1, int k1, float v0, int k0) {
  return v1 > v0 || (v1 == v0 && k1 < k0);
}

// max value, smallest natural index among equals; result broadcast to all
// threads.  One barrier: the scratch slots are next written after at least
// one more barrier (the next block / unit), so no trailing barrier is needed.
__device__ __forceinline__ void block_argmax(float& v, int& k, PeakSlot* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o, 64);
    const int k2 = __shfl_xor(k, o, 64);
    if (better(v2, k2, v, k)) { v = v2; k = k2; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) scratch[w] = PeakSlot{v, k};
  __syncthreads();
  v = scratch[0].v;
  k = scratch[0].k;
#pragma unroll
  for (int i = 1; i < kThreads / 64; i++)
    if (better(scratch[i].v, scratch[i].k, v, k)) { v = scratch[i].v; k = scratch[i].k; }
}

// max over the workgroup, valid in thread 0 only (one barrier, as above)
__device__ __forceinline__ float block_max0(float v, float* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 1; i < kThreads / 64; i++) v = fmaxf(v, scratch[i]);
  }
  return v;
}

// ---- the hot kernel ------------------------------------------------------------
// One workgroup = one work unit: BEST_OF_BLOCKS -> unit = (row, block), the
// statistics of that block go to stats[unit]; NONCOHERENT -> unit = row, |.|^2
// summed over the blocks in registers, stats to stats[row * n_blocks].
// (Row-sized units would leave the last of ~5 rounds of workgroups 1/8 full.)
// Every thread owns radix-31 group t (positions t*31 .. t*31+30) and threads
// t < 496 also own one output of the 16 leftover groups (position 512*31 + t).
template <int MODE, bool DUMP>
__global__ __launch_bounds__(kThreads) void acq_corr_kernel(
    const float2* __restrict__ X, const float2* __restrict__ F, int n_blocks,
    const int* __restrict__ group_code, const int* __restrict__ group_freq, int n_bins,
    int spc, gnsscorr_acq_row* __restrict__ stats, double* __restrict__ dump_power,
    int dump_block, const int* __restrict__ order, const int4* __restrict__ fmap) {
  __shared__ float2 lds[N];
  __shared__ float2 tw[32];
  __shared__ PeakSlot s_pk[kThreads / 64];
  __shared__ float s_mx[kThreads / 64];
  constexpr bool kNonCoh = MODE == GNSSCORR_ACQ_NONCOHERENT;
  ACQ_STAMP(12);
  const int unit = order[blockIdx.x];
  const int rowid = kNonCoh ? unit : unit / n_blocks;
  const int blk0 = kNonCoh ? 0 : unit % n_blocks;
  const int nblk = kNonCoh ? n_blocks : 1;
  const int g = rowid / n_bins, bin = rowid % n_bins;
  const int code = group_code[g];
  const int fid = group_freq[g * n_bins + bin];
  const int4 fm = fmap[fid];
  const Shift sh{fm.y, fm.z, fm.w >> 5, fm.w & 31};
  const int t = threadIdx.x;
  const float inv_n2 = 1.0f / ((float)N * (float)N);
  const bool extra = t < kLeft * 31;
  const int kb = out_base(t);
  // natural index of the leftover output owned by this thread
  const int kx = (out_base(kThreads + t / 31) + (t % 31) * E31) % N;
  init_tw31(tw);

  constexpr int kAcc = kNonCoh ? 32 : 1;
  float pacc[kAcc];
#pragma unroll
  for (int d = 0; d < kAcc; d++) pacc[d] = 0.f;
  float best_pk = -1.f, best_sec = 0.f;
  int best_k = 0;

  const float2* Fc = F + (long)code * NPAD;
  for (int i = 0; i < nblk; i++) {
    const int blk = blk0 + i;
    const float2* Xb = X + ((long)fm.x * n_blocks + blk) * NPAD;
    ACQ_STAMP(i * 6 + 0);
    // D = conj(X) * F  (= conj(X * conj(F)), acquisition.sci:116), then radix-16
    load_mul_pass16(Xb, Fc, lds, t, sh);
    __syncthreads();
    ACQ_STAMP(i * 6 + 1);
    if (!(ACQ_SKIP & 1)) pass33(lds, t);
    __syncthreads();
    ACQ_STAMP(i * 6 + 2);
    float pw[32];  // pw[31] = this thread's leftover output (or -1)
    if (ACQ_SKIP & 2) {
#pragma unroll
      for (int d = 0; d < 32; d++) pw[d] = lds[(t * 31 + d) % N].x;
    } else {
      const float2 y = extra ? dft31_single(lds, tw, t) : make_float2(0.f, 0.f);
      pw[31] = extra ? (y.x * y.x + y.y * y.y) * inv_n2 : -1.f;
      v2f x[31];
#pragma unroll
      for (int d = 0; d < 31; d++) x[d] = ld2(lds[t * 31 + d]);
      dftp<31>(x);
#pragma unroll
      for (int d = 0; d < 31; d++) pw[d] = (x[d].x * x[d].x + x[d].y * x[d].y) * inv_n2;
    }
    ACQ_STAMP(i * 6 + 3);
    if (DUMP && blk == dump_block) {
      int k = kb;
#pragma unroll
      for (int d = 0; d < 31; d++) {
        dump_power[(long)rowid * N + k] = pw[d];
        k += E31;
        if (k >= N) k -= N;
      }
      if (extra) dump_power[(long)rowid * N + kx] = pw[31];
    }
    if (kNonCoh) {
#pragma unroll
      for (int d = 0; d < 32; d++) pacc[d % kAcc] += pw[d];
      __syncthreads();  // LDS is rewritten by the next block
      if (i + 1 < nblk) continue;
#pragma unroll
      for (int d = 0; d < 31; d++) pw[d] = pacc[d % kAcc];
      pw[31] = extra ? pacc[31 % kAcc] : -1.f;
    }
    // Row statistics.  Thread t's 31 strided outputs sit at natural indices
    // kb + 528 d (mod N), so ANY window of < 528 samples holds at most one of
    // them: a per-thread top-2 (max + fmed3) gives the largest value outside
    // the +-spc window without a second pass.  The leftover output (kx) is
    // handled on its own.  Within-thread exact ties keep the first slot
    // (slot order, not natural order).
    if (ACQ_SKIP & 4) {   // diagnostic only: no statistics
      best_pk = pw[0] + pw[30];
      continue;
    }
    float m1 = -1.f, m2 = -1.f;
    int d1 = 0;
#pragma unroll
    for (int d = 0; d < 31; d++) {
      const float v = pw[d];
      d1 = v > m1 ? d : d1;
      m2 = __builtin_amdgcn_fmed3f(m2, m1, v);
      m1 = fmaxf(m1, v);
    }
    int k1 = kb + d1 * E31;
    if (k1 >= N) k1 -= N;
    float v = m1;
    int kk = k1;
    if (extra && better(pw[31], kx, v, kk)) { v = pw[31]; kk = kx; }
    block_argmax(v, kk, s_pk);
    ACQ_STAMP(i * 6 + 4);
    // second peak outside the open window (argmax - spc, argmax + spc), circular
    auto in_win = [&](int k) {
      int dist = k - kk;
      if (dist < 0) dist += N;
      return dist < spc || dist > N - spc;
    };
    float sv = in_win(k1) ? m2 : m1;
    if (extra && !in_win(kx)) sv = fmaxf(sv, pw[31]);
    sv = block_max0(sv, s_mx);
    ACQ_STAMP(i * 6 + 5);
    best_pk = v;
    best_k = kk;
    best_sec = sv;
  }
  if (t == 0) {
    gnsscorr_acq_row r;
    r.peak = best_pk;
    r.argmax = best_k;
    r.second = best_sec;
    r.block = kNonCoh ? -1 : blk0;
    stats[(long)rowid * n_blocks + blk0] = r;
  }
  ACQ_STAMP(13);
}

// ---- the pipelined (persistent, two-role) correlation kernel -------------------
// One workgroup per CU (the 128 KiB row fills the LDS), 1024 threads:
//   waves 0-7  ("compute"): the in-LDS passes of unit u -- 3x11, radix-31 --
//              and the row statistics;
//   waves 8-15 ("stream"):  the HBM/L2 loads, conj(X)*F and radix-16 of unit
//              u+G in registers while the compute waves work, the LDS write
//              of that row once the compute waves hold their radix-31 inputs,
//              and the 16 leftover radix-31 groups of unit u.
// Per unit:  P1 [3x11 | loads+radix-16]  S1  P2 [radix-31 inputs -> regs |
// leftover inputs -> side buffer]  S2  P3 [radix-31 + top-2 | row write +
// leftover outputs]  S3 (argmax)  P4 [second peak]  S4.
// Both roles keep their per-thread working set in the SAME register array r,
// so the stream role's 32 loaded values and the compute role's 31-33 values
// share VGPRs (the 1024-thread launch bound allows 128 per thread).
constexpr int kPipeThreads = 1024;
constexpr int kRole = 512;   // threads per role

template <int O>
__device__ __forceinline__ void dft16_r(v2f (&r)[33]) {
  v2f x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = r[O + i];
  dft16(x);
#pragma unroll
  for (int i = 0; i < 16; i++) r[O + i] = x[i];
}

// conj(X) * F for radix-16 groups g0 = tl and g1 = tl + 512 into r[0..15],
// r[16..31] (8-byte loads: consecutive lanes read consecutive columns, and the
// LDS writes of store16_r are bank-conflict free).  g1 = 1023 (tl = 511) is the
// zero pad column of the HBM rows; it is loaded but never stored.
// Column pairs of the stream role.  A code is real, so its spectrum is
// conjugate-symmetric: F[-k] = conj(F[k]).  Negation acts on the PFA slot
// coordinates one by one ((a, b, c, d) -> (-a, -b, -c, -d), the input map is
// linear), so stream thread tl owns group g = pair_group(tl) and its negative
// neg_group(g): 511 such pairs plus group 0 (self-paired, tl = 511, written
// twice with the same values) cover the 1023 groups, and only the 16 code
// values of g are loaded (acq_symmetrize_kernel makes the stored F exactly
// symmetric, so the derived half equals the stored one bit for bit).
__device__ __forceinline__ int pair_group(int tl) {
  if (tl < 495) return (tl / 15) * 31 + 1 + tl % 15;   // d = 1..15, every (b, c)
  if (tl < 510) {                                      // d = 0, c = 1..5, every b
    const int j = tl - 495;
    return ((j / 5) * 11 + 1 + j % 5) * 31;
  }
  return tl == 510 ? 341 : 0;                          // (1, 0, 0), then group 0
}

__device__ __forceinline__ int neg_group(int g) {
  const int d = g % 31, bc = g / 31, c = bc % 11, b = bc / 11;
  return (((3 - b) % 3) * 11 + (11 - c) % 11) * 31 + (31 - d) % 31;
}

__device__ __forceinline__ void load_mul_r(const float2* __restrict__ Xb,
                                           const float2* __restrict__ Fc, int tl,
                                           const Shift& sh, v2f (&r)[33]) {
  const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)Xb, 0, NPAD * 8, 0x00020000);
  const auto rf = __builtin_amdgcn_make_buffer_rsrc((void*)Fc, 0, NPAD * 8, 0x00020000);
  // tl is made opaque so that the group arithmetic is recomputed per unit
  // instead of being hoisted out of the unit loop
  int t0 = tl;
  asm volatile("" : "+v"(t0));
  const int ga = pair_group(t0), gb = neg_group(ga);
  const int foff = ga * 8;
  // Planes in groups of kLdGroup: all loads of a group are issued before any
  // of its products (sched_group_barrier pins the VMEM reads first), so a
  // unit costs 16 / kLdGroup L2 round trips instead of one per plane.
  // Column ga takes plane a with F[a]; column gb takes plane -a with conj(F[a]).
  constexpr int kLdGroup = ACQ_LDGROUP;
  int x0off = foff, x1off = gb * 8;
  int pa_shift = 0;
  if (!(sh.a == 0 && sh.b == 0 && sh.c == 0 && sh.d == 0)) {   // uniform branch
    x0off = shift_group(ga, sh) * 8;
    x1off = shift_group(gb, sh) * 8;
    pa_shift = sh.a;
  }
#pragma unroll
  for (int a0 = 0; a0 < 16; a0 += kLdGroup) {
    f2v U0[kLdGroup], U1[kLdGroup], F0[kLdGroup];
#pragma unroll
    for (int a = 0; a < kLdGroup; a++) {
      const int an = (16 - (a0 + a)) & 15;
      const int pa = ((a0 + a - pa_shift) & 15) * kPlane * 8;
      const int pn = ((an - pa_shift) & 15) * kPlane * 8;
      const int pf = (a0 + a) * kPlane * 8;
      U0[a] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rx, x0off, pa, 0));
      U1[a] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rx, x1off, pn, 0));
      F0[a] = __builtin_bit_cast(f2v, __builtin_amdgcn_raw_buffer_load_b64(rf, foff, pf, 0));
    }
    __builtin_amdgcn_sched_group_barrier(0x020, 3 * kLdGroup, 0);
#pragma unroll
    for (int a = 0; a < kLdGroup; a++) {
      const int an = (16 - (a0 + a)) & 15;
      const v2f f0 = (v2f){F0[a].x, F0[a].y}, f1 = (v2f){F0[a].x, -F0[a].y};
      r[a0 + a] = bc(U0[a].x) * f0 + bc(U0[a].y) * mul_mi(f0);
      r[16 + an] = bc(U1[a].x) * f1 + bc(U1[a].y) * mul_mi(f1);
    }
  }
  dft16_r<0>(r);
  dft16_r<16>(r);
  // pin the radix-16 results here (P1): without this the arithmetic is sunk
  // past the barriers to its only use, the LDS write in P3
#pragma unroll
  for (int i = 0; i < 32; i++) asm volatile("" : "+v"(r[i]));
}

__device__ __forceinline__ void store16_r(float2* lds, int tl, const v2f (&r)[33]) {
  int t0 = tl;
  asm volatile("" : "+v"(t0));   // per-unit address arithmetic, not hoisted VGPRs
  const int ga = pair_group(t0), gb = neg_group(ga);
#pragma unroll
  for (int a = 0; a < 16; a++) {
    lds[a * M16 + ga] = st2(r[a]);
    lds[a * M16 + gb] = st2(r[16 + a]);
  }
}

// Threads t >= 496 compute a copy of task 0 and store nothing: r is then
// redefined on every lane (a lane that kept its old r would keep it live
// around the whole unit loop).
__device__ __forceinline__ void pass33_r(float2* lds, int t, v2f (&r)[33]) {
  const bool own = t < 16 * 31;
  const int tt = own ? t : 0;
  const int a = tt / 31, d = tt % 31;
  float2* base = lds + a * M16 + d;
#pragma unroll
  for (int i = 0; i < 33; i++) r[i] = ld2(base[i * 31]);
#pragma unroll
  for (int c = 0; c < 11; c++) dft3(r[c], r[11 + c], r[22 + c]);
#pragma unroll
  for (int b = 0; b < 3; b++) {
    v2f x[11];
#pragma unroll
    for (int c = 0; c < 11; c++) x[c] = r[b * 11 + c];
    dftp<11>(x);
#pragma unroll
    for (int c = 0; c < 11; c++) r[b * 11 + c] = x[c];
  }
  if (own) {
#pragma unroll
    for (int i = 0; i < 33; i++) base[i * 31] = st2(r[i]);
  }
}

// Radix-31 of r[0..30] reduced on the fly to this thread's top-2 powers
// |X_d|^2 * scale: the sums/differences overwrite r in place and each output
// pair is squared and folded into (m1, d1, m2) as soon as it exists, so no
// outputs are held (VGPR budget of the 1024-thread kernel).  Slots are visited
// in the order 0, 1, 30, 2, 29, ..., 15, 16; an exact tie keeps the earlier
// visited slot.
__device__ __forceinline__ void top2_push(float p, int d, float& m1, float& m2, int& d1) {
  d1 = p > m1 ? d : d1;
  m2 = __builtin_amdgcn_fmed3f(m2, m1, p);
  m1 = fmaxf(m1, p);
}

__device__ __forceinline__ void dft31_top2(v2f (&r)[33], float scale, float& m1, float& m2,
                                           int& d1) {
  constexpr int P = 31, H = 15;
  const v2f x0 = r[0];
  v2f X0 = x0;
#pragma unroll
  for (int j = 1; j <= H; j++) {
    const v2f s = r[j] + r[P - j], d = r[j] - r[P - j];
    r[j] = s;
    r[P - j] = d;
    X0 += s;
  }
  m1 = (X0.x * X0.x + X0.y * X0.y) * scale;
  m2 = -1.f;
  d1 = 0;
#pragma unroll
  for (int m = 1; m <= H; m++) {
    v2f A = x0, B = (v2f){0.f, 0.f};
#pragma unroll
    for (int j = 1; j <= H; j++) {
      const int q = (j * m) % P;
      A += bc(kCos31[q]) * r[j];
      B += bc(kSin31[q]) * r[P - j];
    }
    // X_m = A - i B and X_{P-m} = A + i B, held as (re_m, re_{P-m}), (im_m, im_{P-m})
    // so that both powers come out of three packed instructions
    const v2f re = __builtin_elementwise_fma(bc(B.y), (v2f){1.f, -1.f}, bc(A.x));
    const v2f im = __builtin_elementwise_fma(bc(B.x), (v2f){-1.f, 1.f}, bc(A.y));
    const v2f pw = __builtin_elementwise_fma(im, im, re * re) * bc(scale);
    top2_push(pw.x, m, m1, m2, d1);
    top2_push(pw.y, P - m, m1, m2, d1);
  }
}

// One output pair (m, 31 - m) -- or X_0 for m = 0 -- of leftover radix-31
// group 512 + g, g = t / 16, m = t % 16, from the side copy of its inputs;
// twiddles from tw16[j][m] = (cos, sin)(2 pi jm / 31), j = 1..15.  Returns the
// pair's top-2 powers and the natural index of the larger.
__device__ __forceinline__ void leftover_pair(const float2* side, const float2* tw16, int t,
                                              float scale, float& m1, float& m2, int& k1) {
  const int g = t >> 4, m = t & 15;
  const float2* x = side + g * 31;
  const v2f x0 = ld2(x[0]);
  v2f A = x0, B = (v2f){0.f, 0.f};
#pragma unroll
  for (int j = 1; j <= 15; j++) {
    const v2f a = ld2(x[j]), b = ld2(x[31 - j]);
    const float2 w = tw16[j * 16 + m];
    A += bc(w.x) * (a + b);
    B += bc(w.y) * (a - b);
  }
  const v2f sb = swp(B);
  const v2f lo = __builtin_elementwise_fma(sb, (v2f){1.f, -1.f}, A);    // X_m
  const v2f hi = __builtin_elementwise_fma(sb, (v2f){-1.f, 1.f}, A);    // X_{31-m}
  const float pl = (lo.x * lo.x + lo.y * lo.y) * scale;
  const float ph = m ? (hi.x * hi.x + hi.y * hi.y) * scale : -1.f;
  const int d1 = ph > pl ? 31 - m : m;
  m1 = fmaxf(pl, ph);
  m2 = fminf(pl, ph);
  k1 = out_base(kThreads + g) + d1 * E31;
  k1 = k1 >= N ? k1 - N : k1;
  k1 = k1 >= N ? k1 - N : k1;
}

// Wave reductions with ds_swizzle (xor 1..16 within each 32-lane half, the
// pattern is an immediate: no per-lane address VGPRs to keep live); the two
// half-wave results go to separate scratch slots.
template <int X>
__device__ __forceinline__ float swz_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v), 0x1f | (X << 10)));
}
template <int X>
__device__ __forceinline__ int swz_i(int v) {
  return __builtin_amdgcn_ds_swizzle(v, 0x1f | (X << 10));
}

__device__ __forceinline__ void pick(float& v, int& k, float v2, int k2) {
  if (better(v2, k2, v, k)) { v = v2; k = k2; }
}

// (v, k) argmax over the workgroup (value max, smallest natural index among
// equals), broadcast to every thread: swizzle steps within 32-lane halves,
// the two halves via readlane, one slot per wave, one barrier, then a
// depth-4 tree over the NT/64 slots.
template <int NT>
__device__ __forceinline__ void block_argmax_n(float& v, int& k, PeakSlot* scratch) {
  pick(v, k, swz_f<1>(v), swz_i<1>(k));
  pick(v, k, swz_f<2>(v), swz_i<2>(k));
  pick(v, k, swz_f<4>(v), swz_i<4>(k));
  pick(v, k, swz_f<8>(v), swz_i<8>(k));
  pick(v, k, swz_f<16>(v), swz_i<16>(k));
  float va = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  int ka = __builtin_amdgcn_readlane(k, 0);
  pick(va, ka, __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32)),
       __builtin_amdgcn_readlane(k, 32));
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = PeakSlot{va, ka};
  __syncthreads();
  constexpr int S = NT / 64;
  float sv[S];
  int sk[S];
#pragma unroll
  for (int i = 0; i < S; i++) { sv[i] = scratch[i].v; sk[i] = scratch[i].k; }
#pragma unroll
  for (int w = 1; w < S; w *= 2)
#pragma unroll
    for (int i = 0; i + w < S; i += 2 * w) pick(sv[i], sk[i], sv[i + w], sk[i + w]);
  v = sv[0];
  k = sk[0];
}

// max over the workgroup, valid in thread 0 only (one barrier)
template <int NT>
__device__ __forceinline__ float block_max0_n(float v, float* scratch) {
  v = fmaxf(v, swz_f<1>(v));
  v = fmaxf(v, swz_f<2>(v));
  v = fmaxf(v, swz_f<4>(v));
  v = fmaxf(v, swz_f<8>(v));
  v = fmaxf(v, swz_f<16>(v));
  const float h = fmaxf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0)),
                        __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32)));
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    constexpr int S = NT / 64;
    float m[S];
#pragma unroll
    for (int i = 0; i < S; i++) m[i] = scratch[i];
#pragma unroll
    for (int w = 1; w < S; w *= 2)
#pragma unroll
      for (int i = 0; i + w < S; i += 2 * w) m[i] = fmaxf(m[i], m[i + w]);
    v = m[0];
  }
  return v;
}

struct UnitInfo {
  int rowid, blk, code;
  int4 fm;
};

__device__ __forceinline__ UnitInfo unit_info(int u, const int* __restrict__ order, int n_blocks,
                                              int n_bins, const int* __restrict__ group_code,
                                              const int* __restrict__ group_freq,
                                              const int4* __restrict__ fmap) {
  UnitInfo ui;
  const int unit = order[u];
  ui.rowid = unit / n_blocks;
  ui.blk = unit % n_blocks;
  const int g = ui.rowid / n_bins, bin = ui.rowid % n_bins;
  ui.code = group_code[g];
  ui.fm = fmap[group_freq[g * n_bins + bin]];
  return ui;
}

// Per-unit statistics of the pipelined kernel, carried across the next
// unit's barriers by the compute role.
struct RowCand {
  float m1, m2, l1, l2;   // own group top-2, leftover pair top-2
  int k1, kl;             // natural indices of m1 / l1
};

// DPP lane exchanges (quad_perm 1032 / 2301, row_half_mirror, row_mirror):
// four steps leave every lane of each 16-lane row holding the row result;
// the four rows are combined through readlane.  Pure VALU, no LDS round trips.
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL>(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float rl_f(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// wave-level (v, k) argmax -> one slot per wave
__device__ __forceinline__ void wave_argmax_slot(float v, int k, PeakSlot* slots) {
  pick(v, k, dpp_f<0xB1>(v), dpp_i<0xB1>(k));
  pick(v, k, dpp_f<0x4E>(v), dpp_i<0x4E>(k));
  pick(v, k, dpp_f<0x141>(v), dpp_i<0x141>(k));
  pick(v, k, dpp_f<0x140>(v), dpp_i<0x140>(k));
  float va = rl_f(v, 0);
  int ka = __builtin_amdgcn_readlane(k, 0);
  pick(va, ka, rl_f(v, 16), __builtin_amdgcn_readlane(k, 16));
  pick(va, ka, rl_f(v, 32), __builtin_amdgcn_readlane(k, 32));
  pick(va, ka, rl_f(v, 48), __builtin_amdgcn_readlane(k, 48));
  if ((threadIdx.x & 63) == 0) slots[threadIdx.x >> 6] = PeakSlot{va, ka};
}

template <int S>
__device__ __forceinline__ PeakSlot read_argmax(const PeakSlot* slots) {
  float sv[S];
  int sk[S];
#pragma unroll
  for (int i = 0; i < S; i++) { sv[i] = slots[i].v; sk[i] = slots[i].k; }
#pragma unroll
  for (int w = 1; w < S; w *= 2)
#pragma unroll
    for (int i = 0; i + w < S; i += 2 * w) pick(sv[i], sk[i], sv[i + w], sk[i + w]);
  return PeakSlot{sv[0], sk[0]};
}

// second-peak candidate of this thread given the row argmax kk (open circular
// window); each candidate set has at most one slot inside any window of < 528
__device__ __forceinline__ float second_cand(const RowCand& c, int kk, int spc) {
  auto in_win = [&](int k) {
    int dist = k - kk;
    if (dist < 0) dist += N;
    return dist < spc || dist > N - spc;
  };
  return fmaxf(in_win(c.k1) ? c.m2 : c.m1, in_win(c.kl) ? c.l2 : c.l1);
}

__device__ __forceinline__ void wave_max_slot(float v, float* slots) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  const float h = fmaxf(fmaxf(rl_f(v, 0), rl_f(v, 16)), fmaxf(rl_f(v, 32), rl_f(v, 48)));
  if ((threadIdx.x & 63) == 0) slots[threadIdx.x >> 6] = h;
}

template <int S>
__device__ __forceinline__ float read_max(const float* slots) {
  float m[S];
#pragma unroll
  for (int i = 0; i < S; i++) m[i] = slots[i];
#pragma unroll
  for (int w = 1; w < S; w *= 2)
#pragma unroll
    for (int i = 0; i + w < S; i += 2 * w) m[i] = fmaxf(m[i], m[i + w]);
  return m[0];
}

__device__ __forceinline__ void write_stats(gnsscorr_acq_row* stats, const UnitInfo& uc,
                                            int n_blocks, float peak, int argmax, float second) {
  gnsscorr_acq_row o;
  o.peak = peak;
  o.argmax = argmax;
  o.second = second;
  o.block = uc.blk;
  stats[(long)uc.rowid * n_blocks + uc.blk] = o;
}

__device__ __forceinline__ gnsscorr_acq_row combine_blocks(const gnsscorr_acq_row* st,
                                                          int n_blocks, int mode) {
  gnsscorr_acq_row r = st[0];
  if (mode != GNSSCORR_ACQ_NONCOHERENT)
    for (int k = 1; k < n_blocks; k++)
      if (!(r.peak > st[k].peak)) r = st[k];
  return r;
}

// one wavefront per group (lane = 0..63); see acq_select_kernel
__device__ void select_group(int g, int lane, const gnsscorr_acq_row* __restrict__ stats,
                             int n_bins, int n_blocks, int mode, int gpr,
                             const int* __restrict__ group_freq,
                             const double* __restrict__ freqs, gnsscorr_acq_row* __restrict__ rows,
                             gnsscorr_acq_result* __restrict__ res) {
  const gnsscorr_acq_row* st = stats + (long)g * n_bins * n_blocks;
  double pk = -1.0;
  int bin = 0x7fffffff;
  for (int b = lane; b < n_bins; b += 64) {
    const gnsscorr_acq_row r = combine_blocks(st + (long)b * n_blocks, n_blocks, mode);
    rows[(long)g * n_bins + b] = r;
    if (r.peak > pk) { pk = r.peak; bin = b; }
  }
  if (!res) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double v2 = __shfl_xor(pk, o, 64);
    const int b2 = __shfl_xor(bin, o, 64);
    if (v2 > pk || (v2 == pk && b2 < bin)) { pk = v2; bin = b2; }
  }
  int cp = 0x7fffffff;
  for (int b = lane; b < n_bins; b += 64) {
    const gnsscorr_acq_row r = combine_blocks(st + (long)b * n_blocks, n_blocks, mode);
    if (r.peak == pk) cp = min(cp, r.argmax);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cp = min(cp, __shfl_xor(cp, o, 64));
  if (lane == 0) {
    const gnsscorr_acq_row rb = combine_blocks(st + (long)bin * n_blocks, n_blocks, mode);
    gnsscorr_acq_result o;
    o.peak = pk;
    o.second = rb.second;
    o.metric = pk / rb.second;
    o.bin = bin;
    o.code_phase = cp + 1;
    // 1 if an exact tie put the global first column in another row than the
    // winning row's own argmax (second peak then centred on the row's argmax)
    o.pad = cp != rb.argmax;
    o.pad2 = 0;
    o.carr_freq = freqs[group_freq[(long)(g % gpr) * n_bins + bin]];   // g: rec * gpr + group
    res[g] = o;
  }
}

__global__ __launch_bounds__(64) void acq_select_kernel(
    const gnsscorr_acq_row* __restrict__ stats, int n_groups, int n_bins, int n_blocks, int mode,
    const int* __restrict__ group_freq, const double* __restrict__ freqs,
    gnsscorr_acq_row* __restrict__ rows, gnsscorr_acq_result* __restrict__ res, int gpr) {
  select_group(blockIdx.x, threadIdx.x, stats, n_bins, n_blocks, mode, gpr, group_freq, freqs,
               rows, res);
}

// BEST_OF_BLOCKS statistics only (unit = (row, block)); launched with at most
// one workgroup per CU, each looping over units u = blockIdx.x + k * gridDim.x.
// Three barriers per unit:
//   P1 [compute: argmax of the previous unit from its slots, its second-peak
//       wave maxima, 3x11 pass | stream: loads + radix-16 of unit u+G]   S1
//   P2 [compute: radix-31 inputs -> regs, leftover inputs -> side copy;
//       thread 0: second peak + stats of the previous unit]              S2
//   P3 [compute: radix-31 + top-2, leftover pair, wave argmax slots |
//       stream: row write of unit u+G]                                   S3
// so the row statistics ride on the next unit's barriers.
__global__ __launch_bounds__(kPipeThreads) void acq_corr_pipe_kernel(
    const float2* __restrict__ X, const float2* __restrict__ F, int n_blocks,
    const int* __restrict__ group_code, const int* __restrict__ group_freq, int n_bins,
    int spc, gnsscorr_acq_row* __restrict__ stats, const int* __restrict__ order,
    const int4* __restrict__ fmap, int n_units) {
  constexpr int S = kRole / 64;   // statistics slots: one per compute wave
  __shared__ float2 lds[N];
  __shared__ float2 side[kLeft * 31];
  __shared__ float2 tw16[16 * 16];
  __shared__ PeakSlot s_pk[S];
  __shared__ float s_mx[S];
  const int t = threadIdx.x;
  // wave-uniform role, made visibly uniform (SGPR) so that the buffer
  // descriptors built inside role branches stay scalar
  const bool stream = __builtin_amdgcn_readfirstlane(t >> 9) != 0;
  const int tl = t & (kRole - 1);
  const int G = gridDim.x;
  const float inv_n2 = 1.0f / ((float)N * (float)N);
  int u = blockIdx.x;
  if (u >= n_units) return;
  if (t < 256) {
    const int j = t >> 4, m = t & 15, q = (j * m) % 31;   // tw16[j][m]: lanes m read 16 consecutive
    tw16[t] = make_float2(kCos31[q], kSin31[q]);
  }
  const int kb = out_base(tl);   // natural index of slot 0 of radix-31 group tl

  v2f r[33];
#pragma unroll
  for (int i = 0; i < 33; i++) r[i] = (v2f){0.f, 0.f};
  if (stream) {   // prologue: the first unit's radix-16 pass
    const UnitInfo un = unit_info(u, order, n_blocks, n_bins, group_code, group_freq, fmap);
    const Shift sh{un.fm.y, un.fm.z, un.fm.w >> 5, un.fm.w & 31};
    load_mul_r(X + ((long)un.fm.x * n_blocks + un.blk) * NPAD, F + (long)un.code * NPAD, tl, sh, r);
    store16_r(lds, tl, r);
  }
  __syncthreads();

  RowCand prev{-1.f, -1.f, -1.f, -1.f, 0, 0};
  PeakSlot pk{-1.f, 0};
  int it = 0;
  for (; u < n_units; u += G, it++) {
    const int un_next = u + G;
    const bool nxt = un_next < n_units;
    ACQ_PSTAMP(it, 0);
    // P1
    if (!stream) {
      if (it > 0) {   // previous unit: row argmax, then second-peak wave maxima
        pk = read_argmax<S>(s_pk);
        wave_max_slot(second_cand(prev, pk.k, spc), s_mx);
      }
      pass33_r(lds, tl, r);
    } else if (nxt) {
      const UnitInfo un = unit_info(un_next, order, n_blocks, n_bins, group_code, group_freq, fmap);
      const Shift sh{un.fm.y, un.fm.z, un.fm.w >> 5, un.fm.w & 31};
      load_mul_r(X + ((long)un.fm.x * n_blocks + un.blk) * NPAD, F + (long)un.code * NPAD, tl, sh, r);
    } else {
#pragma unroll
      for (int i = 0; i < 33; i++) r[i] = (v2f){0.f, 0.f};   // r is redefined on every path
    }
    ACQ_PSTAMP(it, 1);
    __syncthreads();   // S1
    ACQ_PSTAMP(it, 2);
    // P2
    if (!stream) {
#pragma unroll
      for (int d = 0; d < 31; d++) r[d] = ld2(lds[tl * 31 + d]);
      if (tl < kLeft * 31) side[tl] = lds[kThreads * 31 + tl];   // leftover inputs
      if (t == 0 && it > 0)
        write_stats(stats, unit_info(u - G, order, n_blocks, n_bins, group_code, group_freq, fmap),
                    n_blocks, pk.v, pk.k, read_max<S>(s_mx));
    }
    ACQ_PSTAMP(it, 3);
    __syncthreads();   // S2: the row is free
    ACQ_PSTAMP(it, 4);
    // P3: compute role -- radix-31 group tl, then (tl < 256) one output pair of
    // the 16 leftover groups from the side copy; stream role -- the row write
    if (!stream) {
      RowCand c{-1.f, -1.f, -1.f, -1.f, 0, 0};
      int d1;
      dft31_top2(r, inv_n2, c.m1, c.m2, d1);
      c.k1 = kb + d1 * E31;
      if (c.k1 >= N) c.k1 -= N;
      if (tl < kLeft * 16) leftover_pair(side, tw16, tl, inv_n2, c.l1, c.l2, c.kl);
      float v = c.m1;
      int k = c.k1;
      pick(v, k, c.l1, c.kl);
      wave_argmax_slot(v, k, s_pk);
      prev = c;
    } else if (nxt) {
      store16_r(lds, tl, r);
    }
    ACQ_PSTAMP(it, 5);
    __syncthreads();   // S3: next row written, argmax slots complete
    ACQ_PSTAMP(it, 6);
  }
  // epilogue: statistics of the last unit
  if (!stream) {
    pk = read_argmax<S>(s_pk);
    wave_max_slot(second_cand(prev, pk.k, spc), s_mx);
  }
  __syncthreads();
  if (t == 0)
    write_stats(stats, unit_info(u - G, order, n_blocks, n_bins, group_code, group_freq, fmap),
                n_blocks, pk.v, pk.k, read_max<S>(s_mx));
}

// Per group (one wavefront, bins across lanes):
//  combine   acquisition.sci:126-132 -- per bin keep block 1 only if its max
//            is strictly larger than block 2's (generalised: a later block
//            replaces the kept one unless the kept max is strictly larger);
//  select    acquisition.sci:141-186 -- frequencyBinIndex = first row with the
//            largest max, codePhase = first column holding it, metric =
//            peak / second.
// ---- host-side index tables ---------------------------------------------------
static int host_in_index(int p) {
  const int d = p % 31, c = (p / 31) % 11, b = (p / 341) % 3, a = p / 1023;
  return (a * M16 + b * M3 + c * M11 + d * M31) % N;
}
static int host_out_index(int p) {
  const int d = p % 31, c = (p / 31) % 11, b = (p / 341) % 3, a = p / 1023;
  return (int)(((long)a * E16 + (long)b * E3 + (long)c * E11 + (long)d * E31) % N);
}

}  // namespace

// ============================================================================
// context / C ABI
// ============================================================================

static int forward_launch(gnsscorr_acq_ctx* c, const int8_t* src, int iq, int n_blocks,
                          const double* d_freqs, int mode, int n_rows, float2* dst,
                          const double* d_cfreq, const int* d_nrows, int fuse_n = 0);

int acq_grow(void** p, size_t* cap, size_t need, size_t elem) {
  if (need <= *cap) return GNSSCORR_OK;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  HIP_TRY(hipMalloc(p, need * elem));
  *cap = need;
  return GNSSCORR_OK;
}

static int codes_preload(gnsscorr_acq_ctx* c);

extern "C" int gnsscorr_acq_create(gnsscorr_acq_ctx** out, const gnsscorr_acq_cfg* cfg) {
  if (!out || !cfg || cfg->max_freqs < 1 || cfg->max_blocks < 1 || cfg->max_codes < 1 ||
      cfg->samp_rate <= 0 ||
      (cfg->precision != GNSSCORR_ACQ_F64 && cfg->precision != GNSSCORR_ACQ_F32)) {
    gnsscorr_set_error("gnsscorr_acq_create: bad config");
    return GNSSCORR_EINVAL;
  }
  if (cfg->precision == GNSSCORR_ACQ_F32 && cfg->n_samples != N) {
    gnsscorr_set_error("gnsscorr_acq_create: the fp32 path needs n_samples %d (got %d)", N,
                       cfg->n_samples);
    return GNSSCORR_EINVAL;
  }
  if (cfg->precision == GNSSCORR_ACQ_F64 && !acq64_plan_for(cfg->n_samples)) {
    gnsscorr_set_error("gnsscorr_acq_create: n_samples %d outside the fp64 range [64, %d]",
                       cfg->n_samples, 1 << 19);
    return GNSSCORR_EINVAL;
  }
  *out = nullptr;
  // self-check of the prime-factor maps: both must be bijections
  if (cfg->precision == GNSSCORR_ACQ_F32) {
    static int checked = 0;
    if (!checked) {
      char* seen = (char*)calloc(2 * N, 1);
      for (int p = 0; p < N; p++) { seen[host_in_index(p)]++; seen[N + host_out_index(p)]++; }
      for (int i = 0; i < 2 * N; i++)
        if (seen[i] != 1) { free(seen); gnsscorr_set_error("PFA map check failed"); return GNSSCORR_EINVAL; }
      free(seen);
      checked = 1;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gnsscorr_set_error("gnsscorr_acq_create: no HIP device");
    return GNSSCORR_ENODEV;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    gnsscorr_set_error("gnsscorr_acq_create: device %d out of range", cfg->device);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(cfg->device));
  auto* c = new gnsscorr_acq_ctx();
  c->cfg = *cfg;
  c->prec = cfg->precision;
  const int ns = cfg->n_samples;
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, cfg->device) !=
          hipSuccess || c->n_cu < 1)
    c->n_cu = 256;
  if (const char* e = getenv("GNSSCORR_ACQ_PIPE")) c->pipe = atoi(e) != 0;
  auto fail = [&](int code) {
    gnsscorr_acq_destroy(c);
    return code;
  };
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_if, (size_t)ns * 2 * cfg->max_blocks) != hipSuccess ||
      hipMalloc(&c->d_freqs, sizeof(double) * cfg->max_freqs) != hipSuccess ||
      hipMalloc(&c->d_cfreq, sizeof(double) * cfg->max_freqs) != hipSuccess ||
      hipMalloc(&c->d_resid, sizeof(double) * cfg->max_freqs) != hipSuccess ||
      hipMalloc(&c->d_nclass, sizeof(int)) != hipSuccess) {
    gnsscorr_set_error("gnsscorr_acq_create: device allocation failed");
    return fail(GNSSCORR_ENOMEM);
  }
  if (c->prec == GNSSCORR_ACQ_F64) {
    int rc = acq64_init(c);
    if (!rc) rc = acq64_preload(c);
    if (!rc) rc = codes_preload(c);
    if (rc) return fail(rc);
    *out = c;
    return GNSSCORR_OK;
  }
  if (hipMalloc(&c->d_sigma, sizeof(int) * N) != hipSuccess ||
      hipMalloc(&c->d_F, sizeof(float2) * NPAD * (size_t)cfg->max_codes) != hipSuccess ||
      hipMalloc(&c->d_X, sizeof(float2) * NPAD * (size_t)cfg->max_freqs * cfg->max_blocks) != hipSuccess ||
      hipMemset(c->d_F, 0, sizeof(float2) * NPAD * (size_t)cfg->max_codes) != hipSuccess ||
      hipMemset(c->d_X, 0, sizeof(float2) * NPAD * (size_t)cfg->max_freqs * cfg->max_blocks) != hipSuccess ||
      hipMalloc(&c->d_fmap, sizeof(int4) * cfg->max_freqs) != hipSuccess) {
    gnsscorr_set_error("gnsscorr_acq_create: device allocation failed");
    return fail(GNSSCORR_ENOMEM);
  }
  // sigma(p) = n^-1(k(p)): where the forward FFT's output k(p) must be stored
  // so that the correlation kernel reads its input n(p') linearly
  int* inv_in = (int*)malloc(sizeof(int) * N);
  int* sigma = (int*)malloc(sizeof(int) * N);
  for (int p = 0; p < N; p++) inv_in[host_in_index(p)] = p;
  for (int p = 0; p < N; p++) {
    const int q = inv_in[host_out_index(p)];          // LDS position in the correlation kernel
    sigma[p] = (q / M16) * kPlane + q % M16;          // padded HBM index
  }
  hipError_t e = hipMemcpy(c->d_sigma, sigma, sizeof(int) * N, hipMemcpyHostToDevice);
  free(inv_in);
  free(sigma);
  if (e != hipSuccess) {
    gnsscorr_set_error("gnsscorr_acq_create: %s", hipGetErrorString(e));
    return fail(GNSSCORR_EDEVICE);
  }
  if (const int rc = codes_preload(c)) return fail(rc);
  *out = c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_destroy(gnsscorr_acq_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  acq64_free(c);
  void* bufs[] = {c->d_sigma, c->d_F, c->d_X, c->d_if, c->d_freqs, c->d_gcode, c->d_gfreq,
                  c->d_rows, c->d_res, c->d_dump, c->d_order, c->d_stage, c->d_stats,
                  c->d_fmap, c->d_cfreq, c->d_resid, c->d_nclass, c->d_codes8, c->d_chips};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GNSSCORR_OK;
}

// Code spectra are spectra of real sequences; make them exactly
// conjugate-symmetric (F[-k] = conj(F[k]), F real at k = 0 and N/2) so the
// pipelined kernel may derive half of them (pair_group).  Slot s = a*M16 + g
// keeps its value when it precedes its negative and writes the negative.
__global__ __launch_bounds__(256) void acq_symmetrize_kernel(float2* __restrict__ F,
                                                             int n_codes) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n_codes * N) return;
  const int code = (int)(i / N), sl = (int)(i % N);
  const int a = sl / M16, g = sl % M16;
  const int sn = ((16 - a) & 15) * M16 + neg_group(g);
  float2* Fc = F + (long)code * NPAD;
  const float2 v = Fc[a * kPlane + g];
  if (sl == sn)
    Fc[a * kPlane + g] = make_float2(v.x, 0.f);
  else if (sl < sn)
    Fc[(sn / M16) * kPlane + sn % M16] = make_float2(v.x, -v.y);
}

// spectra of the n_codes int8 replicas at d (device), kept resident
static int codes_spectra(gnsscorr_acq_ctx* c, const int8_t* d, int n_codes) {
  if (c->prec == GNSSCORR_ACQ_F64) return acq64_set_codes(c, d, n_codes);
  int rc = forward_launch(c, d, 0, 1, nullptr, 1, n_codes, c->d_F, nullptr, nullptr);
  if (rc) return rc;
  hipLaunchKernelGGL(acq_symmetrize_kernel, dim3((n_codes * N + 255) / 256), dim3(256), 0,
                     c->stream, c->d_F, n_codes);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_set_codes(gnsscorr_acq_ctx* c, int n_codes, const int8_t* h_codes) {
  if (!c || !h_codes || n_codes < 1 || n_codes > c->cfg.max_codes) {
    gnsscorr_set_error("gnsscorr_acq_set_codes: bad arguments (n_codes %d, max %d)", n_codes,
                       c ? c->cfg.max_codes : 0);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const size_t bytes = (size_t)n_codes * c->cfg.n_samples;
  int rc = acq_grow((void**)&c->d_codes8, &c->cap_codes8, bytes, 1);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_codes8, h_codes, bytes, hipMemcpyHostToDevice, c->stream));
  rc = codes_spectra(c, c->d_codes8, n_codes);
  if (rc) return rc;
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->n_codes = n_codes;
  return GNSSCORR_OK;
}

// makeCaTable.sci:64-72 / makeStTable.sci:60-67 on the device: replica sample k
// (1-based) takes chip ceil((ts k) / tc) (1-based; the last sample chip
// codeLength), ts = 1/fs, tc = 1/code_rate, in fp64 exactly as gnsscorr_sample_code
// evaluates it.  One id per replica, passed by value.
constexpr int kIdBatch = 64;
struct CodeIds {
  int id[kIdBatch];
};
__global__ __launch_bounds__(256) void prn_codes_kernel(const int8_t* __restrict__ chips, CodeIds ids,
                                                        int n_ids, int N, double fs,
                                                        int8_t* __restrict__ out) {
  const long total = (long)n_ids * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / N), k = (int)(i % N) + 1;
    const int id = ids.id[r];
    const bool st = id == GNSSCORR_CODE_GLO_ST;
    const int len = st ? 511 : 1023;
    const double ts = 1.0 / fs, tc = 1.0 / (st ? 0.511e6 : 1.023e6);
    long idx = (long)ceil((ts * (double)k) / tc);
    if (k == N) idx = len;
    const long j = ((idx - 1) % len + len) % len;
    out[i] = chips[(st ? 32 : id - 1) * 1023 + j];
  }
}

// Once per context (gnsscorr_acq_create): the chip table (32 C/A codes and the
// ST code), the replica buffer for max_codes codes, and this file's code object
// loaded, so that the context's first set_codes / set_prn_codes costs what
// every later one does.
static int codes_preload(gnsscorr_acq_ctx* c) {
  int8_t h[33 * 1023] = {};
  for (int p = 1; p <= 32; p++) gnsscorr_ca_code(p, h + (p - 1) * 1023);
  gnsscorr_st_code(h + 32 * 1023);
  HIP_TRY(hipMalloc(&c->d_chips, sizeof h));
  HIP_TRY(hipMemcpy(c->d_chips, h, sizeof h, hipMemcpyHostToDevice));
  const int rc = acq_grow((void**)&c->d_codes8, &c->cap_codes8,
                          (size_t)c->cfg.max_codes * c->cfg.n_samples, 1);
  if (rc) return rc;
  hipFuncAttributes a;
  HIP_TRY(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&prn_codes_kernel)));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_set_prn_codes(gnsscorr_acq_ctx* c, int n_codes,
                                          const int32_t* h_code_ids) {
  if (!c || !h_code_ids || n_codes < 1 || n_codes > c->cfg.max_codes) {
    gnsscorr_set_error("gnsscorr_acq_set_prn_codes: bad arguments (n_codes %d, max %d)", n_codes,
                       c ? c->cfg.max_codes : 0);
    return GNSSCORR_EINVAL;
  }
  for (int i = 0; i < n_codes; i++)
    if (h_code_ids[i] < 0 || h_code_ids[i] > 32) {
      gnsscorr_set_error("gnsscorr_acq_set_prn_codes: code id %d (entry %d) is neither a GPS "
                         "PRN 1..32 nor GNSSCORR_CODE_GLO_ST", h_code_ids[i], i);
      return GNSSCORR_EINVAL;
    }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const int n = c->cfg.n_samples;
  int rc = acq_grow((void**)&c->d_codes8, &c->cap_codes8, (size_t)n_codes * n, 1);
  if (rc) return rc;
  for (int b = 0; b < n_codes; b += kIdBatch) {
    CodeIds ids;
    const int nb = n_codes - b < kIdBatch ? n_codes - b : kIdBatch;
    for (int i = 0; i < kIdBatch; i++) ids.id[i] = i < nb ? h_code_ids[b + i] : 1;
    const long total = (long)nb * n;
    const int grid = (int)((total + 255) / 256 < 2048 ? (total + 255) / 256 : 2048);
    hipLaunchKernelGGL(prn_codes_kernel, dim3(grid), dim3(256), 0, c->stream, c->d_chips, ids, nb,
                       n, c->cfg.samp_rate, c->d_codes8 + (size_t)b * n);
    HIP_TRY(hipGetLastError());
  }
  rc = codes_spectra(c, c->d_codes8, n_codes);
  if (rc) return rc;
  c->n_codes = n_codes;
  return GNSSCORR_OK;
}

// XCD-aware workgroup order.  Workgroups are dealt round-robin over the 8
// XCDs (blockIdx % 8 share an L2; MI355X_MICROARCH.md "Workgroup dispatch").
// Rows are cut into tiles of 4 bins x 8 groups (= the 32 CUs of one XCD), so
// the workgroups an XCD runs concurrently read 4 IF-spectrum rows and 8 code
// spectra (~2 MB) from its 4 MB L2 instead of 32 distinct pairs.  Placement
// only changes speed, never results.
static void build_tile_order(int n_groups, int n_bins, int units_per_row, int* perm) {
  const int R = n_groups * n_bins * units_per_row;
  constexpr int TB = 4, TG = 8, NX = 8;
  int* seq = (int*)malloc(sizeof(int) * R);
  int k = 0;
  for (int g0 = 0; g0 < n_groups; g0 += TG)
    for (int b0 = 0; b0 < n_bins; b0 += TB)
      for (int u = 0; u < units_per_row; u++)
        for (int bi = b0; bi < b0 + TB && bi < n_bins; bi++)
          for (int gi = g0; gi < g0 + TG && gi < n_groups; gi++)
            seq[k++] = (gi * n_bins + bi) * units_per_row + u;
  int start[NX + 1];
  start[0] = 0;
  for (int x = 0; x < NX; x++) start[x + 1] = start[x] + (R - x + NX - 1) / NX;
  for (int b = 0; b < R; b++) perm[b] = seq[start[b % NX] + b / NX];
  free(seq);
}

static int ensure_order(gnsscorr_acq_ctx* c, int n_groups, int n_bins, int units_per_row) {
  if (c->d_order && c->order_groups == n_groups && c->order_bins == n_bins &&
      c->order_units == units_per_row)
    return GNSSCORR_OK;
  const int R = n_groups * n_bins * units_per_row;
  int* perm = (int*)malloc(sizeof(int) * R);
  build_tile_order(n_groups, n_bins, units_per_row, perm);
  int rc = acq_grow((void**)&c->d_order, &c->cap_order, R, sizeof(int));
  if (rc) { free(perm); return rc; }
  hipError_t e = hipMemcpyAsync(c->d_order, perm, sizeof(int) * R, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  free(perm);
  if (e != hipSuccess) {
    gnsscorr_set_error("ensure_order: %s", hipGetErrorString(e));
    return GNSSCORR_EDEVICE;
  }
  c->order_groups = n_groups;
  c->order_bins = n_bins;
  c->order_units = units_per_row;
  return GNSSCORR_OK;
}

// forward transform of n_rows rows into dst (padded correlation layout)
static int forward_launch(gnsscorr_acq_ctx* c, const int8_t* src, int iq, int n_blocks,
                          const double* d_freqs, int mode, int n_rows, float2* dst,
                          const double* d_cfreq, const int* d_nrows, int fuse_n) {
  int rc = acq_grow((void**)&c->d_stage, &c->cap_stage, (size_t)n_rows * NPAD, sizeof(float2));
  if (rc) return rc;
  // grid-stride kernels: the device-side class count bounds the work, the grid
  // only the parallelism (n_rows is an upper bound of the rows)
  const int g16 = min(n_rows * ((M16 + kFwd1G - 1) / kFwd1G), 4096);
  const int g1023 = min(n_rows * 16, 1024);
  hipLaunchKernelGGL(acq_fwd16_kernel, dim3(g16),
                     dim3(kFwd1Threads), 0, c->stream, src, iq,
                     n_blocks, d_freqs, 1.0 / c->cfg.samp_rate, mode, c->d_stage, d_cfreq,
                     d_nrows, mode == 0 ? c->coh : 1, n_rows, fuse_n, c->cfg.samp_rate / N,
                     c->d_fmap, c->d_cfreq, c->d_nclass);
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(acq_fwd1023_kernel, dim3(g1023), dim3(kFwd2Threads), 0, c->stream,
                     c->d_stage,
                     c->d_sigma, dst, n_blocks, d_nrows, n_rows);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

static int check_search(gnsscorr_acq_ctx* c, int n_blocks, int n_freqs, int mode) {
  if (n_blocks < 1 || n_blocks * c->coh * c->recs > c->cfg.max_blocks || n_freqs < 1 ||
      n_freqs > c->cfg.max_freqs || c->n_codes < 1 ||
      (mode != GNSSCORR_ACQ_BEST_OF_BLOCKS && mode != GNSSCORR_ACQ_NONCOHERENT)) {
    gnsscorr_set_error("gnsscorr_acq: bad arguments (blocks %d x coherent %d x records %d / "
                       "max_blocks %d, freqs %d/%d, codes %d)", n_blocks, c->coh, c->recs,
                       c->cfg.max_blocks, n_freqs, c->cfg.max_freqs, c->n_codes);
    return GNSSCORR_EINVAL;
  }
  return GNSSCORR_OK;
}

static int spectra_launch(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq, int n_blocks,
                          int n_freqs, const double* d_freqs) {
  int rc = check_search(c, n_blocks, n_freqs, GNSSCORR_ACQ_BEST_OF_BLOCKS);
  if (rc) return rc;
  if (iq & ~(GNSSCORR_IF_IQ | GNSSCORR_IF_PACKED2)) {
    gnsscorr_set_error("gnsscorr_acq: iq must be a set of GNSSCORR_IF_* flags (got %d)", iq);
    return GNSSCORR_EINVAL;
  }
  if (c->prec == GNSSCORR_ACQ_F64) {
    // records are contiguous, so they are recs * n_blocks blocks of one IF
    rc = acq64_spectra(c, d_if, iq, n_blocks * c->recs, n_freqs, d_freqs);
    if (rc) return rc;
    c->spec_blocks = n_blocks;
    c->spec_recs = c->recs;
    c->spec_freqs = n_freqs;
    return GNSSCORR_OK;
  }
  // spectrum classes on the fs/N grid (one forward FFT per class and block)
  const int fuse = n_freqs <= kFuseClass ? n_freqs : 0;
  if (!fuse) {
    const size_t cls_lds =
        n_freqs <= kClassLds ? (size_t)((n_freqs + 1) & ~1) * 8 + (size_t)n_freqs * 16 : 0;
    hipLaunchKernelGGL(acq_classify_kernel, dim3(1), dim3(1024), cls_lds, c->stream, d_freqs,
                       n_freqs, c->cfg.samp_rate / N, c->d_fmap, c->d_cfreq, c->d_nclass,
                       c->d_resid);
    HIP_TRY(hipGetLastError());
  }
  rc = forward_launch(c, d_if, iq, n_blocks, d_freqs, 0, n_freqs * n_blocks, c->d_X, c->d_cfreq,
                      c->d_nclass, fuse);
  if (rc) return rc;
  c->spec_blocks = n_blocks;
  c->spec_freqs = n_freqs;
  return GNSSCORR_OK;
}

static int correlate_launch(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_groups, int n_bins,
                            const double* d_freqs, const int32_t* d_gcode,
                            const int32_t* d_gfreq, int spc, gnsscorr_acq_row* d_rows,
                            gnsscorr_acq_result* d_res, double* d_dump, int dump_block) {
  int rc = check_search(c, n_blocks, c->spec_freqs > 0 ? c->spec_freqs : 1, mode);
  if (rc) return rc;
  if (n_groups < 1 || n_bins < 1 || spc < 1 || spc > c->cfg.n_samples / 2 ||
      n_blocks != c->spec_blocks ||
      (c->prec == GNSSCORR_ACQ_F64 && c->spec_recs != c->recs)) {
    gnsscorr_set_error("gnsscorr_acq_correlate: bad arguments (groups %d, bins %d, spc %d, "
                       "blocks %d vs spectra %d)", n_groups, n_bins, spc, n_blocks, c->spec_blocks);
    return GNSSCORR_EINVAL;
  }
  const int upr = mode == GNSSCORR_ACQ_NONCOHERENT ? 1 : n_blocks;  // work units per row
  // records: every group on every record (virtual groups), or with a per-group
  // record table each group on its own record only
  const int nrec = c->prec == GNSSCORR_ACQ_F64 && !c->d_group_rec ? c->spec_recs : 1;
  if (c->d_group_rec && (c->prec != GNSSCORR_ACQ_F64 || c->plan64 == 3 || d_dump)) {
    gnsscorr_set_error("gnsscorr_acq_correlate: per-group records need a compiled fp64 plan");
    return GNSSCORR_EINVAL;
  }
  const int gall = n_groups * nrec;   // virtual groups rec * n_groups + g
  rc = ensure_order(c, gall, n_bins, upr);
  if (rc) return rc;
  rc = acq_grow((void**)&c->d_stats, &c->cap_stats, (size_t)gall * n_bins * n_blocks,
            sizeof(gnsscorr_acq_row));
  if (rc) return rc;
  const int n_units = n_groups * n_bins * upr;
  if (c->prec == GNSSCORR_ACQ_F64) {
    rc = acq64_correlate(c, n_blocks, mode, n_groups, n_bins, d_gcode, d_gfreq, spc, d_dump,
                         dump_block);
    if (rc) return rc;
  } else {
#define ACQ_CORR_LAUNCH(M, D)                                                                \
  hipLaunchKernelGGL((acq_corr_kernel<M, D>), dim3(n_units), dim3(kThreads), 0, c->stream,    \
                     c->d_X, c->d_F, n_blocks, d_gcode, d_gfreq, n_bins, spc, c->d_stats,      \
                     d_dump, dump_block, c->d_order, c->d_fmap)
  if (d_dump)
    ACQ_CORR_LAUNCH(GNSSCORR_ACQ_BEST_OF_BLOCKS, true);
  else if (mode == GNSSCORR_ACQ_NONCOHERENT)
    ACQ_CORR_LAUNCH(GNSSCORR_ACQ_NONCOHERENT, false);
  else if (c->pipe) {
    hipLaunchKernelGGL(acq_corr_pipe_kernel, dim3(n_units < c->n_cu ? n_units : c->n_cu),
                       dim3(kPipeThreads), 0, c->stream, c->d_X, c->d_F, n_blocks, d_gcode,
                       d_gfreq, n_bins, spc, c->d_stats, c->d_order, c->d_fmap, n_units);
  } else
    ACQ_CORR_LAUNCH(GNSSCORR_ACQ_BEST_OF_BLOCKS, false);
#undef ACQ_CORR_LAUNCH
  HIP_TRY(hipGetLastError());
  }
  c->stat_groups = n_groups;
  c->stat_recs = nrec;
  c->stat_bins = n_bins;
  c->stat_blocks = n_blocks;
  c->stat_mode = mode;
  if (d_rows || d_res) {
    if (!d_rows || (d_res && !d_freqs)) {
      gnsscorr_set_error("gnsscorr_acq_correlate: d_res needs d_rows and d_freqs");
      return GNSSCORR_EINVAL;
    }
    hipLaunchKernelGGL(acq_select_kernel, dim3(gall), dim3(64), 0, c->stream, c->d_stats,
                       gall, n_bins, n_blocks, mode, d_gfreq, d_freqs, d_rows, d_res, n_groups);
    HIP_TRY(hipGetLastError());
  }
  return GNSSCORR_OK;
}

static int search_launch(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq, int n_blocks, int mode,
                         int n_freqs, const double* d_freqs, int n_groups, int n_bins,
                         const int32_t* d_gcode, const int32_t* d_gfreq, int spc,
                         gnsscorr_acq_row* d_rows, gnsscorr_acq_result* d_res, double* d_dump,
                         int dump_block) {
  int rc = spectra_launch(c, d_if, iq, n_blocks, n_freqs, d_freqs);
  if (rc) return rc;
  return correlate_launch(c, n_blocks, mode, n_groups, n_bins, d_freqs, d_gcode, d_gfreq, spc,
                          d_rows, d_res, d_dump, dump_block);
}

extern "C" int gnsscorr_acq_spectra_dev(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq,
                                        int n_blocks, int n_freqs, const double* d_freqs) {
  if (!c || !d_if || !d_freqs) {
    gnsscorr_set_error("gnsscorr_acq_spectra_dev: null argument");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  return spectra_launch(c, d_if, iq, n_blocks, n_freqs, d_freqs);
}

extern "C" int gnsscorr_acq_correlate_dev(gnsscorr_acq_ctx* c, int n_blocks, int mode,
                                          const double* d_freqs, int n_groups, int n_bins,
                                          const int32_t* d_group_code,
                                          const int32_t* d_group_freq, int spc,
                                          gnsscorr_acq_row* d_rows, gnsscorr_acq_result* d_res) {
  if (!c || !d_group_code || !d_group_freq || (d_res && (!d_freqs || !d_rows))) {
    gnsscorr_set_error("gnsscorr_acq_correlate_dev: null argument");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  return correlate_launch(c, n_blocks, mode, n_groups, n_bins, d_freqs, d_group_code,
                          d_group_freq, spc, d_rows, d_res, nullptr, -1);
}

extern "C" int gnsscorr_acq_select_dev(gnsscorr_acq_ctx* c, int n_groups, int n_bins,
                                       const double* d_freqs, const int32_t* d_group_freq,
                                       gnsscorr_acq_row* d_rows, gnsscorr_acq_result* d_res) {
  if (!c || !d_freqs || !d_group_freq || !d_rows || n_groups != c->stat_groups ||
      n_bins != c->stat_bins || n_groups < 1) {
    gnsscorr_set_error("gnsscorr_acq_select_dev: bad arguments (shape must match the last "
                       "correlate call: %d groups x %d bins)", c ? c->stat_groups : 0,
                       c ? c->stat_bins : 0);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const int gall = n_groups * c->stat_recs;
  hipLaunchKernelGGL(acq_select_kernel, dim3(gall), dim3(64), 0, c->stream, c->d_stats, gall,
                     n_bins, c->stat_blocks, c->stat_mode, d_group_freq, d_freqs, d_rows, d_res,
                     n_groups);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_search_dev(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq,
                                       int n_blocks, int mode, int n_freqs, const double* d_freqs,
                                       int n_groups, int n_bins, const int32_t* d_group_code,
                                       const int32_t* d_group_freq, int spc,
                                       gnsscorr_acq_row* d_rows, gnsscorr_acq_result* d_res) {
  if (!c || !d_if || !d_freqs || !d_group_code || !d_group_freq || !d_rows) {
    gnsscorr_set_error("gnsscorr_acq_search_dev: null argument");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  return search_launch(c, d_if, iq, n_blocks, mode, n_freqs, d_freqs, n_groups, n_bins,
                       d_group_code, d_group_freq, spc, d_rows, d_res, nullptr, -1);
}

static int stage_host(gnsscorr_acq_ctx* c, const int8_t* h_if, int iq, int n_blocks, int n_freqs,
                      const double* h_freqs, int n_groups, int n_bins, const int32_t* h_gcode,
                      const int32_t* h_gfreq) {
  if (n_blocks < 1 || n_blocks * c->coh * c->recs > c->cfg.max_blocks || n_freqs < 1 ||
      n_freqs > c->cfg.max_freqs) {
    gnsscorr_set_error("gnsscorr_acq_search: n_blocks (x coherent ms x records) / n_freqs "
                       "outside the context capacity");
    return GNSSCORR_EINVAL;
  }
  for (int g = 0; g < n_groups; g++) {
    if (h_gcode[g] < 0 || h_gcode[g] >= c->n_codes) {
      gnsscorr_set_error("gnsscorr_acq_search: group %d code %d not uploaded", g, h_gcode[g]);
      return GNSSCORR_EINVAL;
    }
    for (int b = 0; b < n_bins; b++) {
      const int f = h_gfreq[(long)g * n_bins + b];
      if (f < 0 || f >= n_freqs) {
        gnsscorr_set_error("gnsscorr_acq_search: group %d bin %d freq index %d invalid", g, b, f);
        return GNSSCORR_EINVAL;
      }
    }
  }
  const size_t R = (size_t)n_groups * n_bins;
  int rc;
  if ((rc = acq_grow((void**)&c->d_rows, &c->cap_rows, R * c->recs, sizeof(gnsscorr_acq_row))))
    return rc;
  if ((rc = acq_grow((void**)&c->d_res, &c->cap_res, (size_t)n_groups * c->recs,
                     sizeof(gnsscorr_acq_result))))
    return rc;
  if ((rc = acq_grow((void**)&c->d_gcode, &c->cap_gcode, n_groups, sizeof(int)))) return rc;
  if ((rc = acq_grow((void**)&c->d_gfreq, &c->cap_gfreq, R, sizeof(int)))) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_if, h_if,
                         (size_t)if_bytes((int64_t)c->recs * n_blocks * c->coh * c->cfg.n_samples *
                                              ((iq & GNSSCORR_IF_IQ) ? 2 : 1),
                                          iq & GNSSCORR_IF_PACKED2),
                         hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_freqs, h_freqs, sizeof(double) * n_freqs, hipMemcpyHostToDevice,
                         c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_gcode, h_gcode, sizeof(int) * n_groups, hipMemcpyHostToDevice,
                         c->stream));
  HIP_TRY(hipMemcpyAsync(c->d_gfreq, h_gfreq, sizeof(int) * R, hipMemcpyHostToDevice, c->stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_search(gnsscorr_acq_ctx* c, const int8_t* h_if, int iq, int n_blocks,
                                   int mode, int n_freqs, const double* h_freqs, int n_groups,
                                   int n_bins, const int32_t* h_group_code,
                                   const int32_t* h_group_freq, int spc,
                                   gnsscorr_acq_row* h_rows, gnsscorr_acq_result* h_res) {
  if (!c || !h_if || !h_freqs || !h_group_code || !h_group_freq || n_groups < 1 || n_bins < 1) {
    gnsscorr_set_error("gnsscorr_acq_search: bad arguments");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  int rc = stage_host(c, h_if, iq, n_blocks, n_freqs, h_freqs, n_groups, n_bins, h_group_code,
                      h_group_freq);
  if (rc) return rc;
  rc = search_launch(c, c->d_if, iq, n_blocks, mode, n_freqs, c->d_freqs, n_groups, n_bins,
                     c->d_gcode, c->d_gfreq, spc, c->d_rows, c->d_res, nullptr, -1);
  if (rc) return rc;
  const int nro = c->d_group_rec ? 1 : c->recs;   // per-group records: one result per group
  if (h_rows)
    HIP_TRY(hipMemcpyAsync(h_rows, c->d_rows,
                           sizeof(gnsscorr_acq_row) * nro * n_groups * n_bins,
                           hipMemcpyDeviceToHost, c->stream));
  if (h_res)
    HIP_TRY(hipMemcpyAsync(h_res, c->d_res, sizeof(gnsscorr_acq_result) * nro * n_groups,
                           hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_power_row(gnsscorr_acq_ctx* c, const int8_t* h_if, int iq,
                                      int n_blocks, int block, double freq, int code,
                                      double* h_power) {
  if (!c || !h_if || !h_power || block < 0 || block >= n_blocks || code < 0 ||
      code >= c->n_codes) {
    gnsscorr_set_error("gnsscorr_acq_power_row: bad arguments");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const int32_t gc = code, gf = 0;
  const int recs = c->recs;   // one record, whatever set_records says
  const int32_t* grec = c->d_group_rec;   // and no per-group records
  c->recs = 1;
  c->d_group_rec = nullptr;
  int rc = stage_host(c, h_if, iq, n_blocks, 1, &freq, 1, 1, &gc, &gf);
  if (!rc && !c->d_dump && hipMalloc(&c->d_dump, sizeof(double) * c->cfg.n_samples) != hipSuccess) {
    gnsscorr_set_error("gnsscorr_acq_power_row: out of device memory");
    rc = GNSSCORR_ENOMEM;
  }
  if (!rc)
    rc = search_launch(c, c->d_if, iq, n_blocks, GNSSCORR_ACQ_BEST_OF_BLOCKS, 1, c->d_freqs, 1,
                       1, c->d_gcode, c->d_gfreq, 16, c->d_rows, nullptr, c->d_dump, block);
  c->recs = recs;
  c->d_group_rec = grec;
  c->spec_blocks = 0;   // its one-record spectra must not serve a later multi-record correlate
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(h_power, c->d_dump, sizeof(double) * c->cfg.n_samples,
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_set_coherent(gnsscorr_acq_ctx* c, int coh_ms) {
  if (!c || coh_ms < 1 || coh_ms > c->cfg.max_blocks) {
    gnsscorr_set_error("gnsscorr_acq_set_coherent: need 1 <= coh_ms <= max_blocks");
    return GNSSCORR_EINVAL;
  }
  c->coh = coh_ms;
  c->spec_blocks = 0;   // resident spectra were made with the previous setting
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_set_group_records(gnsscorr_acq_ctx* c, const int32_t* d_group_rec) {
  if (!c) return GNSSCORR_EINVAL;
  if (d_group_rec && (c->prec != GNSSCORR_ACQ_F64 || c->plan64 == 3)) {
    gnsscorr_set_error("gnsscorr_acq_set_group_records: needs the fp64 precision and a compiled "
                       "plan (N = 16368 or 16000)");
    return GNSSCORR_EINVAL;
  }
  // the caller keeps it alive; values outside [0, records) are clamped into that range
  // by the correlation kernel, and set_records drops the table
  c->d_group_rec = d_group_rec;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_set_records(gnsscorr_acq_ctx* c, int n_records) {
  if (!c || n_records < 1 || n_records > c->cfg.max_blocks) {
    gnsscorr_set_error("gnsscorr_acq_set_records: need 1 <= n_records <= max_blocks");
    return GNSSCORR_EINVAL;
  }
  // the generic engine takes records on its mixed-radix / four-step plans (the units of
  // every record in one chunk loop), not on Bluestein's
  if (n_records > 1 && (c->prec != GNSSCORR_ACQ_F64 || (c->plan64 == 3 && !c->mix_nr))) {
    gnsscorr_set_error("gnsscorr_acq_set_records: several records per search need the fp64 "
                       "precision and a compiled plan (n_samples %d or %d) or a mixed-radix "
                       "generic plan (no prime factor above 31)", 16368, 16000);
    return GNSSCORR_EINVAL;
  }
  // a per-group record table was made for the previous record count: set it again
  if (n_records != c->recs) c->d_group_rec = nullptr;
  c->recs = n_records;
  c->spec_blocks = 0;   // resident spectra were made with the previous setting
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_acq_sync(gnsscorr_acq_ctx* c) {
  if (!c) return GNSSCORR_EINVAL;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" void* gnsscorr_acq_stream(gnsscorr_acq_ctx* c) { return c ? (void*)c->stream : nullptr; }
