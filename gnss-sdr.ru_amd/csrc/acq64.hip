// acq64.hip -- parallel code-phase acquisition at the reference's precision
// (fp64), on gfx950.
//
// Reference: POSTPROCESSING_SCILAB_RECEIVERS/GPS/L1/acquisition.sci:46-192
// (GLONASS: GLONASS/L1/acquisition.sci:46-198), which Scilab evaluates in
// doubles:  X = fft(exp(i f 2 pi t) .* block), |ifft(X .* conj(fft(code)))|^2,
// keep the block with the larger maximum, then peak / code phase / second
// peak outside +-1 chip.  This file computes every one of those steps in fp64
// (wipe-off, forward transforms, products, inverse transform, powers and the
// comparisons), so rows agree with an fp64 evaluation to ~1e-13 relative.
//
// MI355X design
//  * A 1-ms row of N complex doubles (256 KiB at N = 16368) does not fit the
//    160 KiB LDS, so it lives in REGISTERS: T threads hold ~N/T complex values
//    each, and every FFT stage is a batch of small in-register DFTs.  Between
//    stages the row is exchanged through LDS in two halves -- the real parts
//    (N doubles = 128 KiB), then the imaginary parts -- so the LDS only ever
//    holds one fp64 plane of the row.
//  * Three stages N = R1 * R2 * R3 per plan, two exchanges per transform:
//      N = 16368 (16.368 Msps, BASELINE config 2): 16 x 33 x 31, Good-Thomas
//        prime-factor (pairwise coprime): no twiddles at all; the Ruritanian
//        input map and the CRT output map are folded into addressing, and the
//        spectra are stored pre-permuted so the hot loads stay coalesced;
//        512 threads, the 16 radix-31 groups beyond 512 are done as direct
//        31-term sums from a side copy;
//      N = 16000 (16 Msps, the Scilab receivers' initSettings.sci:69 default):
//        40 x 40 x 10 Cooley-Tukey (decimation in frequency), 400 threads,
//        every stage balanced (40 values per thread); inter-stage twiddles
//        W^(k m) are generated per group from one table load by a complex
//        recurrence (error ~1e-15).
//  * Small DFTs are compile-time compositions: symmetric prime kernels
//    (X_m = A_m - i B_m, X_{P-m} = A_m + i B_m), Good-Thomas for coprime
//    splits (33 = 3 x 11, 40 = 8 x 5, 10 = 2 x 5), Cooley-Tukey for prime
//    powers (16 = 4 x 4, 8 = 2 x 4); twiddle constants are constexpr-evaluated.
//  * The inverse FFT is a forward FFT of conj(Y): |ifft(Y)|^2 = |fft(conj Y)|^2 / N^2.
//  * The correlation kernel fuses conj(X)*F (with the bin's circular shift on
//    the fs/N grid folded into the X load), the three stages, |.|^2, the
//    non-coherent sum over blocks, and exact row statistics (argmax = first
//    natural index of the maximum; second peak = max outside the open circular
//    window (argmax - spc, argmax + spc)) in two register passes.
#include <hip/hip_runtime.h>
#include <limits.h>
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

// Diagnostic hook: tools/acq64_stamps.hip defines ACQ64_STAMP(i) to record
// s_memtime at the barriers of the correlation kernel; nothing in the library.
#ifndef ACQ64_STAMP
#define ACQ64_STAMP(i)
#endif

namespace {

typedef double v2d __attribute__((ext_vector_type(2)));

// ---- compile-time arithmetic -------------------------------------------------
constexpr double kPi = 3.14159265358979323846264338327950288;

// LDS one workgroup may allocate on the build's offload arch: the library is
// built for gfx950 only (Makefile ARCH), where a workgroup may take the CU's
// whole 160 KiB.  acq64_corr_kernel sizes its parked non-coherent sums from it.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "acq64.hip sizes its LDS for gfx950 (160 KiB per workgroup)"
#endif
constexpr int kLdsBudget = 160 * 1024;

constexpr double poly_sin(double x) {   // |x| <= pi/4, 1 ulp
  double x2 = x * x, term = x, sum = x;
  for (int i = 1; i < 12; i++) {
    term *= -x2 / (double)((2 * i) * (2 * i + 1));
    sum += term;
  }
  return sum;
}
constexpr double poly_cos(double x) {
  double x2 = x * x, term = 1.0, sum = 1.0;
  for (int i = 1; i < 12; i++) {
    term *= -x2 / (double)((2 * i - 1) * (2 * i));
    sum += term;
  }
  return sum;
}
struct CS { double c, s; };
// cos, sin of 2 pi j / R: exact octant reduction in integers, then a series
constexpr CS cs2pi(long j, long R) {
  j %= R;
  if (j < 0) j += R;
  const long q = (8 * j) / R, rem = 8 * j - q * R;   // angle = (q + rem/R) pi/4
  double c = 0, s = 0;
  if ((q & 1) == 0) {
    const double x = (double)rem / (double)R * (kPi / 4);
    c = poly_cos(x);
    s = poly_sin(x);
  } else {   // phi = pi/4 + x in [pi/4, pi/2): use pi/2 - phi = (R - rem)/R pi/4
    const double y = (double)(R - rem) / (double)R * (kPi / 4);
    c = poly_sin(y);
    s = poly_cos(y);
  }
  switch ((q >> 1) & 3) {
    case 0: return CS{c, s};
    case 1: return CS{-s, c};
    case 2: return CS{-c, -s};
    default: return CS{s, -c};
  }
}
template <int R>
struct TwTab {
  double c[R], s[R];
  constexpr TwTab() : c{}, s{} {
    for (int j = 0; j < R; j++) {
      const CS v = cs2pi(j, R);
      c[j] = v.c;
      s[j] = v.s;
    }
  }
};
template <int R>
constexpr TwTab<R> kTw{};

constexpr int cgcd(int a, int b) { return b == 0 ? a : cgcd(b, a % b); }
constexpr int cinv(int a, int m) {   // a^-1 mod m (gcd(a, m) = 1)
  a %= m;
  for (int x = 1; x < m; x++)
    if ((long)a * x % m == 1) return x;
  return m == 1 ? 0 : -1;
}
constexpr bool is_prime(int r) {
  if (r < 2) return false;
  for (int d = 2; d * d <= r; d++)
    if (r % d == 0) return false;
  return true;
}
constexpr int small_pf(int r) {
  for (int d = 2; d * d <= r; d++)
    if (r % d == 0) return d;
  return r;
}
// largest power of the smallest prime factor dividing r
constexpr int pf_power(int r) {
  const int p = small_pf(r);
  int q = 1;
  while (r % (q * p) == 0) q *= p;
  return q;
}

// ---- complex helpers -----------------------------------------------------------
__device__ __forceinline__ v2d mul_mi(v2d v) { return (v2d){v.y, -v.x}; }   // -i v
__device__ __forceinline__ v2d mul_pi(v2d v) { return (v2d){-v.y, v.x}; }   // +i v
__device__ __forceinline__ v2d cmul(v2d a, v2d b) {
  return (v2d){fma(a.x, b.x, -(a.y * b.y)), fma(a.x, b.y, a.y * b.x)};
}
// v * W_R^j, W = exp(-2 pi i / R); j is a compile-time constant after unrolling
template <int R>
__device__ __forceinline__ v2d twc(v2d v, int j) {
  j %= R;
  if (j == 0) return v;
  if (4 * j == R) return mul_mi(v);
  if (2 * j == R) return -v;
  if (4 * j == 3 * R) return mul_pi(v);
  const double c = kTw<R>.c[j], s = kTw<R>.s[j];   // W^j = c - i s
  return (v2d){fma(v.x, c, v.y * s), fma(v.y, c, -(v.x * s))};
}

// ---- small in-register DFTs (forward, natural order in and out) ---------------
template <int R>
__device__ __forceinline__ void dft(v2d (&x)[R]);

__device__ __forceinline__ void dft2(v2d (&x)[2]) {
  const v2d a = x[0], b = x[1];
  x[0] = a + b;
  x[1] = a - b;
}
__device__ __forceinline__ void dft4(v2d (&x)[4]) {
  const v2d t0 = x[0] + x[2], t1 = x[0] - x[2], t2 = x[1] + x[3], t3 = x[1] - x[3];
  x[0] = t0 + t2;
  x[2] = t0 - t2;
  x[1] = t1 + mul_mi(t3);
  x[3] = t1 + mul_pi(t3);
}
// symmetric prime-length DFT
template <int P>
__device__ __forceinline__ void dft_prime(v2d (&x)[P]) {
  constexpr int H = (P - 1) / 2;
  v2d s[H + 1], d[H + 1];
#pragma unroll
  for (int j = 1; j <= H; j++) {
    s[j] = x[j] + x[P - j];
    d[j] = x[j] - x[P - j];
  }
  const v2d x0 = x[0];
  v2d X0 = x0;
#pragma unroll
  for (int j = 1; j <= H; j++) X0 += s[j];
#pragma unroll
  for (int m = 1; m <= H; m++) {
    v2d A = x0, B = (v2d){0.0, 0.0};
#pragma unroll
    for (int j = 1; j <= H; j++) {
      const int q = (j * m) % P;
      const double c = kTw<P>.c[q], sn = kTw<P>.s[q];
      A = (v2d){fma(c, s[j].x, A.x), fma(c, s[j].y, A.y)};
      B = (v2d){fma(sn, d[j].x, B.x), fma(sn, d[j].y, B.y)};
    }
    x[m] = (v2d){A.x + B.y, A.y - B.x};       // A - i B
    x[P - m] = (v2d){A.x - B.y, A.y + B.x};   // A + i B
  }
  x[0] = X0;
}
// symmetric prime DFT fused with |.|^2 * scale: put(k, |X_k|^2 scale) for every
// output k.  Outputs are folded into the powers as each (m, P-m) pair is
// formed, so the complex outputs are never all live (register pressure of the
// non-coherent kernel, whose running sums stay live across the transform).
// symmetric prime DFT that hands each output to emit(k, X_k) as its (m, P-m) pair
// is formed (s_j, d_j in place in x): the 31 complex outputs are never all live
// SERIAL: one output pair at a time (a scheduling barrier after each): the compiler
// otherwise interleaves all (P-1)/2 accumulator pairs, 4 P more live registers
template <int P, bool SERIAL = false, class Emit>
__device__ __forceinline__ void dft_prime_emit(v2d (&x)[P], const Emit& emit) {
  constexpr int H = (P - 1) / 2;
#pragma unroll
  for (int j = 1; j <= H; j++) {
    const v2d a = x[j], b = x[P - j];
    x[j] = a + b;        // s_j
    x[P - j] = a - b;    // d_j
  }
  v2d X0 = x[0];
#pragma unroll
  for (int j = 1; j <= H; j++) X0 += x[j];
#pragma unroll
  for (int m = 1; m <= H; m++) {
    v2d A = x[0], B = (v2d){0.0, 0.0};
#pragma unroll
    for (int j = 1; j <= H; j++) {
      const int q = (j * m) % P;
      const double c = kTw<P>.c[q], sn = kTw<P>.s[q];
      A = (v2d){fma(c, x[j].x, A.x), fma(c, x[j].y, A.y)};
      B = (v2d){fma(sn, x[P - j].x, B.x), fma(sn, x[P - j].y, B.y)};
    }
    emit(m, (v2d){A.x + B.y, A.y - B.x});       // A - iB
    emit(P - m, (v2d){A.x - B.y, A.y + B.x});   // A + iB
    if constexpr (SERIAL) __builtin_amdgcn_sched_barrier(0);
  }
  emit(0, X0);
}
template <int P, class Put>
__device__ __forceinline__ void dft_prime_power(v2d (&x)[P], const Put& put_power, double scale) {
  dft_prime_emit<P>(x, [&](int k, v2d v) { put_power(k, fma(v.x, v.x, v.y * v.y) * scale); });
}

// Good-Thomas R = A * B, gcd(A, B) = 1: n = (a B + b A) mod R, k = CRT(ka, kb)
template <int A, int B>
__device__ __forceinline__ void dft_pfa(v2d (&x)[A * B]) {
  constexpr int R = A * B;
  constexpr int eA = B * cinv(B % A, A) % R, eB = A * cinv(A % B, B) % R;
  v2d y[A][B];
#pragma unroll
  for (int a = 0; a < A; a++)
#pragma unroll
    for (int b = 0; b < B; b++) y[a][b] = x[(a * B + b * A) % R];
#pragma unroll
  for (int b = 0; b < B; b++) {
    v2d t[A];
#pragma unroll
    for (int a = 0; a < A; a++) t[a] = y[a][b];
    dft<A>(t);
#pragma unroll
    for (int a = 0; a < A; a++) y[a][b] = t[a];
  }
#pragma unroll
  for (int a = 0; a < A; a++) dft<B>(y[a]);
#pragma unroll
  for (int a = 0; a < A; a++)
#pragma unroll
    for (int b = 0; b < B; b++) x[(a * eA + b * eB) % R] = y[a][b];
}
// Cooley-Tukey R = A * B (decimation in frequency): n = a B + b, k = ka + A kb
template <int A, int B>
__device__ __forceinline__ void dft_ct(v2d (&x)[A * B]) {
  constexpr int R = A * B;
  v2d y[A][B];
#pragma unroll
  for (int b = 0; b < B; b++) {
    v2d t[A];
#pragma unroll
    for (int a = 0; a < A; a++) t[a] = x[a * B + b];
    dft<A>(t);
#pragma unroll
    for (int a = 0; a < A; a++) y[a][b] = twc<R>(t[a], a * b);
  }
#pragma unroll
  for (int a = 0; a < A; a++) dft<B>(y[a]);
#pragma unroll
  for (int a = 0; a < A; a++)
#pragma unroll
    for (int b = 0; b < B; b++) x[a + A * b] = y[a][b];
}
template <int R>
__device__ __forceinline__ void dft(v2d (&x)[R]) {
  if constexpr (R == 1) {
  } else if constexpr (R == 2) {
    dft2(x);
  } else if constexpr (R == 4) {
    dft4(x);
  } else if constexpr (is_prime(R)) {
    dft_prime<R>(x);
  } else if constexpr (pf_power(R) != R) {
    constexpr int A = pf_power(R);
    dft_pfa<A, R / A>(x);
  } else {
    constexpr int A = (small_pf(R) == 2 && R >= 16) ? 4 : small_pf(R);
    dft_ct<A, R / A>(x);
  }
}

// ---- plans -----------------------------------------------------------------------
// N = R1 R2 R3.  Positions between stages (same for both kinds):
//   after stage 1: k1*G1 + g,       g = n2*R3 + n3   (G1 = R2*R3 = stage-1 groups)
//   after stage 2: (k1*R2 + k2)*R3 + n3
// stage 2 groups g2 = k1*R3 + n3 (G2 = R1*R3), stage 3 groups g3 = k1*R2 + k2.
// PFA: input n = (n1 Q1 + n2 Q2 + n3 Q3) mod N, output k = (k1 E1 + k2 E2 + k3 E3) mod N,
//      spectra stored at n1*G1 + n2*R3 + n3 (digits n_i = (n mod R_i) INV_i mod R_i).
// CT:  input n = n1*G1 + n2*R3 + n3, output k = k1 + R1 k2 + R1 R2 k3, twiddles
//      W_N^(k1 g) after stage 1 and W_G1^(k2 n3) after stage 2; natural storage.
template <int N_, int R1_, int R2_, int R3_, int T_, bool PFA_>
struct Plan {
  static constexpr int N = N_, R1 = R1_, R2 = R2_, R3 = R3_, T = T_;
  static constexpr bool PFA = PFA_;
  static constexpr int TB = (T + 63) / 64 * 64;   // launched threads (whole waves)
  static constexpr int NW = TB / 64;
  static constexpr int G1 = N / R1, G2 = N / R2, G3 = N / R3;
  static constexpr int K1 = (G1 + T - 1) / T, K2 = (G2 + T - 1) / T;
  static constexpr int K3 = G3 / T, L = G3 - K3 * T;   // leftover stage-3 groups
  static constexpr int LS = L * R3 > 0 ? L * R3 : 1;
  // LDS exchange layouts.  PFA plans (PlanA) keep the natural positions.  Cooley-Tukey
  // plans pad them so that every exchange read and write is free of bank conflicts
  // (PlanB at natural positions: 46 % of its LDS cycles were conflicts, PMC
  // profiles/r6/pmc_gps_scilab_r6d.json):
  //  exchange 1: stage-1 output (k1, g) at k1 LG1 + g.  Stage-2 group g2 = t reads
  //    (t / R3) LG1 + t % R3 + n2 R3: with LG1 = R3 (mod 32) a 32-lane ds_read_b64 group
  //    hits the double banks t + c (mod 32), all distinct; the writes are runs of g.
  //  exchange 2: (k1, k2, n3) at k1 LB2 + k2 + n3 S3 (S3 = R2 + 1: injective).  The
  //    writes (fixed k2, lanes (t / R3, t % R3)) hit S3 t (mod 16) with S3 odd; the
  //    stage-3 reads (fixed n3, lanes k1 = t / R3, k2 = t % R3 + R3 j) hit LB2 (t / R3)
  //    + t % R3 = t (mod 32) with LB2 = R3 (mod 32).
  //  (MI355X_MICROARCH.md LDS table: ds_read_b64 2 x 32 lanes, bank (a/4) mod 64;
  //  ds_write_b64 4 x 16 lanes, bank (a/4) mod 32.)
  static constexpr int pad_to(int v, int m, int r) { return v + (((r - v) % m) + m) % m; }
  static constexpr int LG1 = PFA_ ? N / R1 : pad_to(N / R1, 32, R3);
  static constexpr int S2 = PFA_ ? R3 : 1;
  static constexpr int S3 = PFA_ ? 1 : pad_to(R2 + 1, 8, 1) | 1;
  static constexpr int LB2 = PFA_ ? R2 * R3 : pad_to(R2 * S2 + (R3 - 1) * S3 + 1, 32, R3);
  static constexpr int LX = PFA_ ? N : (R1 * LG1 > R1 * LB2 ? R1 * LG1 : R1 * LB2);
  static constexpr int Q1 = N / R1, Q2 = N / R2, Q3 = N / R3;
  static constexpr int INV1 = PFA ? cinv(Q1 % R1, R1) : 0;
  static constexpr int INV2 = PFA ? cinv(Q2 % R2, R2) : 0;
  static constexpr int INV3 = PFA ? cinv(Q3 % R3, R3) : 0;
  static constexpr int E1 = PFA ? (int)((long)Q1 * INV1 % N) : 0;
  static constexpr int E2 = PFA ? (int)((long)Q2 * INV2 % N) : 0;
  static constexpr int E3 = PFA ? (int)((long)Q3 * INV3 % N) : 0;
  static_assert(R1 * R2 * R3 == N, "plan factors");
  static_assert(L * R3 <= T, "leftover stage-3 inputs must fit one per thread");
  // leftover stage-3 groups run as symmetric tasks (group, m), m = 0..(R3-1)/2:
  // task t computes outputs m and R3-m (m > 0) of group K3*T + t % L
  static constexpr int LT = L * ((R3 + 1) / 2);
  static_assert(LT <= T, "leftover tasks must fit one per thread");
  __device__ static __forceinline__ bool lvalid(int t, int j) {
    return t < LT && (j == 0 || t >= L);
  }
  __device__ static __forceinline__ int lslot(int t, int j) {
    return j == 0 ? t / L : R3 - t / L;
  }
  static_assert(!PFA || (cgcd(R1, R2) == 1 && cgcd(R1, R3) == 1 && cgcd(R2, R3) == 1),
                "PFA needs coprime factors");
  // Code spectra are spectra of real sequences, F[-k] = conj(F[k]).  In PFA
  // digits negation is digit-wise, so with two stage-1 groups per thread a
  // thread can own a group and its negative and load F once for both:
  // SYM plans pair the 1023 radix-16 groups as (g, -g) -- 511 pairs + group 0.
  static constexpr bool SYM = PFA && K1 == 2 && R2 == 33 && R3 == 31 && T == 512;
  // stage-3 group of main slot j of thread t.  CT plans with several groups
  // per thread give a thread groups (k1, k2 + j R2/K3) so that ALL its outputs
  // (natural k1 + R1 k2 + R1 R2 k3) lie at least N/(R3 K3) apart.
  __device__ static __forceinline__ int group3(int t, int j) {
    if constexpr (!PFA && K3 > 1 && L == 0 && R2 % K3 == 0 && T == R1 * (R2 / K3)) {
      constexpr int W = R2 / K3;
      return (t / W) * R2 + t % W + W * j;
    } else {
      return t + j * T;
    }
  }
  // a thread's main stage-3 outputs are at least this far apart (circularly):
  // any window of fewer samples holds at most one of them
  static constexpr int SPACING =
      (!PFA && K3 > 1 && L == 0 && R2 % K3 == 0 && T == R1 * (R2 / K3)) ? N / (R3 * K3)
                                                                      : (K3 == 1 ? N / R3 : 1);
  // stage-1 group of slot j of thread t (SYM: the pair (g, -g)), -1 if none
  __device__ static __forceinline__ int group1(int t, int j) {
    if constexpr (SYM) {
      // slot 0 takes whole rows n2 = 1..16 (every n3) and row 0's n3 = 1..15;
      // the mirrors (rows 32..17, row 0's n3 = 30..16) are slot 1.  A wave's
      // slot-0 (and slot-1) groups are then ~2 consecutive 31-group rows:
      // each of its 16-byte loads covers ~1 KB of contiguous storage
      // (circularly shifted by the bin), not ~5 runs of 15 groups
      int g;
      if (t < 496) g = (1 + t / R3) * R3 + t % R3;    // n2 = 1..16, n3 = 0..30
      else if (t < 511) g = t - 495;                  // n2 = 0, n3 = 1..15
      else g = t == 511 ? 0 : -1;                     // group 0 pairs with itself
      if (j == 0 || g <= 0) return j == 0 ? g : -1;
      const int n2 = g / R3, n3 = g % R3;
      return ((R2 - n2) % R2) * R3 + (R3 - n3) % R3;
    } else {
      const int g = t + j * T;
      return (t < T && g < G1) ? g : -1;
    }
  }
  // natural input index of stage-1 element (n1, g)
  __device__ static __forceinline__ int in_index(int n1, int g) {
    if constexpr (PFA) {
      const int n2 = g / R3, n3 = g % R3;
      int n = n1 * Q1 + n2 * Q2;          // < 2N
      n -= n >= N ? N : 0;
      n += n3 * Q3;                        // < 2N
      return n >= N ? n - N : n;
    } else {
      return n1 * G1 + g;
    }
  }
  // natural output index of stage-3 slot k3 of group g3: base + k3*step (mod N)
  __device__ static __forceinline__ void out_base(int g3, int& base, int& step) {
    const int k1 = g3 / R2, k2 = g3 % R2;
    if constexpr (PFA) {
      base = (k1 * E1 + k2 * E2) % N;      // < R1*N + R2*N < 2^31
      step = E3;
    } else {
      base = k1 + R1 * k2;
      step = R1 * R2;
    }
  }
  // storage position of stage-3 output k3 of group g3: sbase(g3) + soff(k3).
  // PFA: the natural index k = CRT(k1, k2, k3) has k mod R_i = k_i, so its
  // storage digits are k_i * INV_i mod R_i -- no division per value.
  __device__ static __forceinline__ int sbase(int g3) {
    const int k1 = g3 / R2, k2 = g3 % R2;
    if constexpr (PFA) return (k1 * INV1 % R1) * G1 + (k2 * INV2 % R2) * R3;
    else return k1 + R1 * k2;
  }
  static constexpr int soff(int k3) { return PFA ? (k3 * INV3 % R3) : R1 * R2 * k3; }
  // storage position of natural index k in a spectrum row
  __device__ static __forceinline__ int store_index(int k) {
    if constexpr (PFA) {
      const int n1 = (k % R1) * INV1 % R1, n2 = (k % R2) * INV2 % R2, n3 = (k % R3) * INV3 % R3;
      return n1 * G1 + n2 * R3 + n3;
    } else {
      return k;
    }
  }
};
static_assert((long)16 * 15345 + (long)33 * 16368 < (1L << 31), "int index maps");

typedef Plan<16368, 16, 33, 31, 512, true> PlanA;   // 16.368 Msps
typedef Plan<16000, 40, 40, 10, 400, false> PlanB;  // 16 Msps

// multiply x[k] (k = 1..R-1) by w^k, w = W_M^m from the table; two interleaved
// recurrences (odd / even powers) halve the dependency chain
template <int R>
__device__ __forceinline__ void twiddle_run(v2d (&x)[R], v2d w) {
  const v2d w2 = cmul(w, w);
  v2d po = w, pe = w2;
#pragma unroll
  for (int k = 1; k < R; k++) {
    if (k & 1) {
      x[k] = cmul(x[k], po);
      if (k + 2 < R) po = cmul(po, w2);
    } else {
      x[k] = cmul(x[k], pe);
      if (k + 2 < R) pe = cmul(pe, w2);
    }
  }
}

__device__ __forceinline__ double part(v2d v, int p) { return p ? v.y : v.x; }
__device__ __forceinline__ void set_part(v2d& v, int p, double d) {
  if (p)
    v.y = d;
  else
    v.x = d;
}

// The transform from stage-1 inputs v1 (loaded by the caller) to stage-3
// outputs v3 (main groups g3 = t + j*T) and vl[j] (leftover outputs where
// P::lvalid(t, j): slot P::lslot(t, j) of group K3*T + t % L).  lds: N doubles; side: the
// LS real parts of the leftover groups' stage-3 inputs (their imaginary parts stay in
// the plane after exchange 2: the leftover tasks read lds[K3*T*R3 ..] after fft_core's
// last barrier, so a caller that writes the plane next must pass a barrier first);
// twN: W_N^j (global, CT plans only).
// Keeps the exchange reads as single ds_read_b64 (256 B/clk per CU): the
// load/store optimizer otherwise pairs them into ds_read2_b64, which the LDS
// serves at 128 B/clk (MI355X_MICROARCH.md, LDS table).
__device__ __forceinline__ void lds_read_fence() { __builtin_amdgcn_sched_barrier(0); }

// the lane id by mbcnt, opaque to the compiler (recomputed where it is used,
// never hoisted or kept live across a loop)
__device__ __forceinline__ int lane_id_opaque() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

struct NoHook {
  __device__ void operator()() const {}
};
template <class P, class Hook = NoHook, bool kStage3 = true, bool kPinStage1 = false>
__device__ __forceinline__ void fft_core(double* lds, double* side,
                                         const v2d* __restrict__ twN, int t,
                                         v2d (&v1)[P::K1][P::R1], v2d (&v3)[P::K3][P::R3],
                                         v2d (&vl)[2], const Hook& before_exchange = Hook()) {
  constexpr int R1 = P::R1, R2 = P::R2, R3 = P::R3, T = P::T, G2 = P::G2;
  const bool act = t < T;
  // ---- stage 1
#pragma unroll
  for (int j = 0; j < P::K1; j++) {
    dft<R1>(v1[j]);
    if constexpr (!P::PFA) {
      const int g = P::group1(t, j);
      if (g >= 0) twiddle_run<R1>(v1[j], twN[g]);
    }
  }
  if constexpr (kPinStage1) {
    // stage 1 completes before the hook: its results pass through empty asm
    // statements, the hook's loads stay behind a compiler memory barrier
#pragma unroll
    for (int j = 0; j < P::K1; j++)
#pragma unroll
      for (int k = 0; k < R1; k++) asm volatile("" : "+v"(v1[j][k].x), "+v"(v1[j][k].y));
    asm volatile("" ::: "memory");
  }
  before_exchange();   // the caller may still use the LDS up to here
  // ---- exchange 1: re then im
  v2d v2[P::K2][R2];
#pragma unroll
  for (int p = 0; p < 2; p++) {
#pragma unroll
    for (int j = 0; j < P::K1; j++) {
      const int g = P::group1(t, j);
      if (g >= 0) {
#pragma unroll
        for (int k1 = 0; k1 < R1; k1++) lds[k1 * P::LG1 + g] = part(v1[j][k1], p);
      }
    }
    __syncthreads();
    ACQ64_STAMP(1 + 2 * p);
#pragma unroll
    for (int j = 0; j < P::K2; j++) {
      const int g2 = t + j * T;
      if (act && g2 < G2) {
        const int base = (g2 / R3) * P::LG1 + g2 % R3;
#pragma unroll
        for (int n2 = 0; n2 < R2; n2++) {
          set_part(v2[j][n2], p, lds[base + n2 * R3]);
          lds_read_fence();
        }
      }
    }
    __syncthreads();
    ACQ64_STAMP(2 + 2 * p);
  }
  // ---- stage 2
#pragma unroll
  for (int j = 0; j < P::K2; j++) {
    dft<R2>(v2[j]);
    if constexpr (!P::PFA) {
      const int g2 = t + j * T;
      if (act && g2 < G2) twiddle_run<R2>(v2[j], twN[(g2 % R3) * R1]);   // W_G1^n3 = W_N^(n3 R1)
    }
  }
  // ---- exchange 2
#pragma unroll
  for (int p = 0; p < 2; p++) {
#pragma unroll
    for (int j = 0; j < P::K2; j++) {
      const int g2 = t + j * T;
      if (act && g2 < G2) {
        const int k1 = g2 / R3, n3 = g2 % R3;
#pragma unroll
        for (int k2 = 0; k2 < R2; k2++) lds[k1 * P::LB2 + k2 * P::S2 + n3 * P::S3] = part(v2[j][k2], p);
      }
    }
    __syncthreads();
    ACQ64_STAMP(5 + 2 * p);
#pragma unroll
    for (int j = 0; j < P::K3; j++) {
      const int g3 = act ? P::group3(t, j) : 0;
      const int b3 = (g3 / R2) * P::LB2 + (g3 % R2) * P::S2;
#pragma unroll
      for (int n3 = 0; n3 < R3; n3++) {
        set_part(v3[j][n3], p, lds[b3 + n3 * P::S3]);
        lds_read_fence();
      }
    }
    if constexpr (P::L > 0) {
      // PFA layout: leftover group K3*T + lg, input n3 at (K3*T + lg)*R3 + n3
      static_assert(P::PFA, "leftover groups assume the PFA exchange layout");
      if (p == 0 && t < P::L * R3) side[t] = lds[P::K3 * T * R3 + t];
    }
    __syncthreads();
    ACQ64_STAMP(6 + 2 * p);
  }
  // ---- stage 3 (main groups: left to the caller when !kStage3)
  if constexpr (kStage3) {
#pragma unroll
    for (int j = 0; j < P::K3; j++) dft<R3>(v3[j]);
  }
  if constexpr (P::L > 0) {
    // leftover groups: the symmetric prime DFT (dft_prime) split by output
    // pair, real parts from the side copy, imaginary parts from the plane
    // (exchange 2's last phase), W^(jm) from the constant table kTw (cos, -sin;
    // an LDS copy took the 400 B that the non-coherent kernel's sums need)
    if (t < P::LT) {
      constexpr int H = (R3 - 1) / 2;
      const int lg = t % P::L, m = t / P::L;
      const double* xr = side + lg * R3;
      const double* xi = lds + P::K3 * T * R3 + lg * R3;
      v2d A = (v2d){xr[0], xi[0]}, B = (v2d){0.0, 0.0};
      int q = m;
#pragma unroll
      for (int j = 1; j <= H; j++) {
        const v2d a = (v2d){xr[j], xi[j]}, b = (v2d){xr[R3 - j], xi[R3 - j]};
        const v2d w = (v2d){kTw<R3>.c[q], -kTw<R3>.s[q]};
        const v2d sj = a + b, dj = a - b;
        A = (v2d){fma(w.x, sj.x, A.x), fma(w.x, sj.y, A.y)};
        B = (v2d){fma(-w.y, dj.x, B.x), fma(-w.y, dj.y, B.y)};
        q += m;
        q -= q >= R3 ? R3 : 0;
      }
      vl[0] = (v2d){A.x + B.y, A.y - B.x};   // A - iB
      vl[1] = (v2d){A.x - B.y, A.y + B.x};   // A + iB (slot R3 - m)
    }
  }
}

// ---- workgroup reductions --------------------------------------------------------
// Wave step: DPP row_shr 1/2/4/8 (a Hillis-Steele scan inside each 16-lane row,
// the identity shifted in) leaves each row's result in its lane 15; the four
// rows combine in scalar registers.  VALU only: no ds_bpermute round trips
// (a 64-bit __shfl_xor is two LDS-crossbar operations per step).  Every lane
// of the wave must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double ident, double v) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(ident), __double2loint(v), CTRL, 0xF,
                                             0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(ident), __double2hiint(v), CTRL, 0xF,
                                             0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ bool better(double v1, int k1, double v0, int k0) {
  return v1 > v0 || (v1 == v0 && k1 < k0);
}
template <int CTRL>
__device__ __forceinline__ void argmax_step(double& v, int& k) {
  const double v2 = dpp_f64<CTRL>(-1.0, v);
  const int k2 = __builtin_amdgcn_update_dpp(INT_MAX, k, CTRL, 0xF, 0xF, false);
  if (better(v2, k2, v, k)) { v = v2; k = k2; }
}
// argmax (largest value, first index on ties) of the wave; uniform result
__device__ __forceinline__ void wave_argmax(double& v, int& k) {
  argmax_step<0x111>(v, k);
  argmax_step<0x112>(v, k);
  argmax_step<0x114>(v, k);
  argmax_step<0x118>(v, k);
  double bv = readlane_f64(v, 15);
  int bk = __builtin_amdgcn_readlane(k, 15);
#pragma unroll
  for (int r = 31; r < 64; r += 16) {
    const double v2 = readlane_f64(v, r);
    const int k2 = __builtin_amdgcn_readlane(k, r);
    if (better(v2, k2, bv, bk)) { bv = v2; bk = k2; }
  }
  v = bv;
  k = bk;
}
__device__ __forceinline__ double wave_max(double v) {   // values >= -1
  v = fmax(v, dpp_f64<0x111>(-1.0, v));
  v = fmax(v, dpp_f64<0x112>(-1.0, v));
  v = fmax(v, dpp_f64<0x114>(-1.0, v));
  v = fmax(v, dpp_f64<0x118>(-1.0, v));
  return fmax(fmax(readlane_f64(v, 15), readlane_f64(v, 31)),
              fmax(readlane_f64(v, 47), readlane_f64(v, 63)));
}
// tid: the caller's thread index (default threadIdx.x)
template <int NW>
__device__ __forceinline__ void block_argmax(double& v, int& k, double* sv, int* sk,
                                             int tid = threadIdx.x) {
  wave_argmax(v, k);
  if ((tid & 63) == 0) { sv[tid >> 6] = v; sk[tid >> 6] = k; }
  __syncthreads();
  v = sv[0];
  k = sk[0];
#pragma unroll
  for (int i = 1; i < NW; i++)
    if (better(sv[i], sk[i], v, k)) { v = sv[i]; k = sk[i]; }
}
template <int NW>
__device__ __forceinline__ double block_max0(double v, double* sm, int tid = threadIdx.x) {
  v = wave_max(v);
  if ((tid & 63) == 0) sm[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int i = 1; i < NW; i++) v = fmax(v, sm[i]);
  }
  return v;
}

// ---- forward transforms ------------------------------------------------------------
// Inputs are written in the plan's storage order (element n at store_index(n)),
// so the forward FFT reads its stage-1 groups with coalesced loads at constant
// offsets, exactly like the correlation kernel reads the spectra.
// IF rows: x[n] = sum_{p<coh} IF[blk][n + pN] * exp(i f ((n+pN)*2)*pi*ts), evaluated as
// acquisition.sci:61-62,107 does (phasePoints = (0:L-1)*2*%pi*ts; exp(%i*f*phasePoints))
// at the class frequency f = cfreq[cls]; row = cls * n_blocks + blk.  With
// fuse_n > 0 (short frequency tables) every workgroup first classifies the
// table itself (acq64_classify_kernel's job) and workgroup 0 publishes it.
constexpr int kFuseClass = 64;
__device__ __forceinline__ double grid_residue(double f, double delta) {
  double r = fmod(f, delta);
  return r < 0 ? r + delta : r;
}
template <class P>
__global__ __launch_bounds__(256) void acq64_wipe_kernel(
    const int8_t* __restrict__ src, int iq, int n_blocks, int coh, const double* __restrict__ cfreq_in,
    const int* __restrict__ n_cls_dev, double ts, v2d* __restrict__ out, int fuse_n,
    const double* __restrict__ freqs, double delta, int2* __restrict__ fmap_out,
    double* __restrict__ cfreq_out, int* __restrict__ nclass_out) {
  constexpr int N = P::N;
  __shared__ double s_r[kFuseClass], s_cf[kFuseClass];
  __shared__ int s_l[kFuseClass], s_nc;
  const double* cfreq = cfreq_in;
  int n_cls;
  if (fuse_n > 0) {
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
        int mN = fabs(q) < 1e9 ? (int)fmod(q, (double)N) : 0;
        mN += mN < 0 ? N : 0;
        fmap_out[t] = make_int2(cls, mN);
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
    n_cls = s_nc;
  } else {
    n_cls = *n_cls_dev;
  }
  const long total = (long)n_cls * n_blocks * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / N), n = (int)(i % N);
    const int cls = row / n_blocks, blk = row % n_blocks;
    // (an LDS / global pointer select would make this a flat load)
    const double f = fuse_n > 0 ? s_cf[cls] : cfreq[cls];
    const bool cplx = iq & GNSSCORR_IF_IQ, pk = iq & GNSSCORR_IF_PACKED2;
    const int ne = cplx ? 2 : 1;
    const long e0 = (long)blk * coh * N * ne;   // first element of the block
    double re = 0.0, im = 0.0;
    for (int p = 0; p < coh; p++) {
      const long m = n + (long)p * N;
      const double I = (double)if_elem(src, e0 + ne * m, pk);
      const double Q = cplx ? (double)if_elem(src, e0 + 2 * m + 1, pk) : 0.0;
      const double th = f * ((((double)m * 2.0) * M_PI) * ts);
      double sn, cs;
      sincos(th, &sn, &cs);
      re += I * cs - Q * sn;
      im += I * sn + Q * cs;
    }
    out[(long)row * N + P::store_index(n)] = (v2d){re, im};
  }
}

template <class P>
__global__ __launch_bounds__(256) void acq64_codes_kernel(const int8_t* __restrict__ codes,
                                                          long n, v2d* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i - i % P::N + P::store_index((int)(i % P::N))] = (v2d){(double)codes[i], 0.0};
}

// Rows in storage order -> spectra in storage order.
template <class P>
__global__ __launch_bounds__(P::TB) void acq64_fwd_kernel(const v2d* __restrict__ in,
                                                          const int* __restrict__ n_cls_dev,
                                                          int per_cls, int n_rows,
                                                          v2d* __restrict__ out, int rs,
                                                          const v2d* __restrict__ twN) {
  __shared__ double lds[P::LX];
  __shared__ double side[P::LS];
  const int t = threadIdx.x;
  // rows grid-strided over a capped grid (n_rows is an upper bound of the
  // rows when the class count is on the device); fft_core ends on a barrier
  // after its last exchange read, but the leftover tasks (P::L > 0) read the
  // plane after it: the next row's exchange-1 writes wait for a barrier
  const int rows = n_cls_dev ? *n_cls_dev * per_cls : n_rows;
  for (int w = blockIdx.x; w < rows; w += gridDim.x) {
    const v2d* src = in + (long)w * P::N;
    v2d v1[P::K1][P::R1];
#pragma unroll
    for (int j = 0; j < P::K1; j++) {
      const int g0 = P::group1(t, j), g = g0 < 0 ? 0 : g0;
#pragma unroll
      for (int n1 = 0; n1 < P::R1; n1++) v1[j][n1] = src[n1 * P::G1 + g];
    }
    v2d v3[P::K3][P::R3], vl[2] = {(v2d){0.0, 0.0}, (v2d){0.0, 0.0}};
    fft_core<P>(lds, side, twN, t, v1, v3, vl);
    v2d* o = out + (long)w * rs;
    if (t < P::T) {
#pragma unroll
      for (int j = 0; j < P::K3; j++) {
        const int sb = P::sbase(P::group3(t, j));
#pragma unroll
        for (int k3 = 0; k3 < P::R3; k3++) o[sb + P::soff(k3)] = v3[j][k3];
      }
    }
    if constexpr (P::L > 0) {
#pragma unroll
      for (int j = 0; j < 2; j++)
        if (P::lvalid(t, j)) {
          int base, step;
          P::out_base(P::K3 * P::T + t % P::L, base, step);
          o[P::store_index((base + P::lslot(t, j) * step) % P::N)] = vl[j];
        }
      __syncthreads();   // leftover tasks' plane reads before the next row's writes
    }
  }
}

// ---- forward transforms of prime-factor plans in two launches --------------------
// Stage 1 (radix R1 over the G1 groups) in place: element n1*G1 + g of a row
// becomes k1*G1 + g -- each thread reads and writes the same R1 positions.
template <class P>
__global__ __launch_bounds__(256) void acq64_fwd1_kernel(v2d* __restrict__ io,
                                                         const int* __restrict__ n_cls_dev,
                                                         int per_cls, int n_rows) {
  // grid-stride: the launch is sized for the host's upper bound on the rows
  // (classes <= frequencies), capped; the actual count is read here
  const int rows = n_cls_dev ? *n_cls_dev * per_cls : n_rows;
  const long total = (long)rows * P::G1;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int row = (int)(i / P::G1), g = (int)(i % P::G1);
    v2d* r = io + (long)row * P::N;
    v2d v[P::R1];
#pragma unroll
    for (int n1 = 0; n1 < P::R1; n1++) v[n1] = r[n1 * P::G1 + g];
    dft<P::R1>(v);
#pragma unroll
    for (int k1 = 0; k1 < P::R1; k1++) r[k1 * P::G1 + g] = v[k1];
  }
}

// Stages 2 and 3 of one (row, k1): the G1 = R2 x R3 values k1*G1 + n2*R3 + n3
// are an independent R2 x R3 prime-factor transform.  One output per thread
// as direct DFT sums (R2, then R3 complex MACs) through LDS; the results go to
// the plan's storage positions sbase(k1*R2 + k2) + soff(k3).
constexpr int kFwd23Threads = 1024;
template <class P>
__global__ __launch_bounds__(kFwd23Threads) void acq64_fwd23_kernel(
    const v2d* __restrict__ in, const int* __restrict__ n_cls_dev, int per_cls, int n_rows,
    v2d* __restrict__ out, int rs) {
  constexpr int R2 = P::R2, R3 = P::R3, G1 = P::G1;
  static_assert(G1 <= kFwd23Threads, "one output per thread");
  __shared__ v2d s_a[G1], s_b[G1];
  __shared__ v2d w2[R2], w3[R3];
  // grid-stride over (row, k1) (see acq64_fwd1_kernel)
  const int rows = n_cls_dev ? *n_cls_dev * per_cls : n_rows;
  const int t = threadIdx.x;
  if (t < R2) w2[t] = (v2d){kTw<R2>.c[t], -kTw<R2>.s[t]};
  if (t < R3) w3[t] = (v2d){kTw<R3>.c[t], -kTw<R3>.s[t]};
  for (int u = blockIdx.x; u < rows * P::R1; u += gridDim.x) {
  const int row = u / P::R1, k1 = u % P::R1;
  if (t < G1) s_a[t] = in[(long)row * P::N + k1 * G1 + t];
  __syncthreads();
  // (four partial sums: the latency of one dependent chain, not the FMA
  // rate, bounds these single-wave-per-SIMD sums)
  if (t < G1) {   // stage 2: output (k2, n3) = sum_n2 a[n2][n3] W_R2^(n2 k2)
    const int k2 = t / R3, n3 = t % R3;
    v2d acc[4] = {(v2d){0.0, 0.0}, (v2d){0.0, 0.0}, (v2d){0.0, 0.0}, (v2d){0.0, 0.0}};
    // W^(n2 k2) by recurrence from one table read (a per-lane gather of the
    // table at every step conflicts in LDS); error ~R2 ulp
    const v2d wk = w2[k2];
    v2d w = (v2d){1.0, 0.0};
#pragma unroll
    for (int n2 = 0; n2 < R2; n2++) {
      acc[n2 & 3] += cmul(s_a[n2 * R3 + n3], w);
      w = cmul(w, wk);
    }
    s_b[t] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();
  if (t < G1) {   // stage 3: output (k2, k3) = sum_n3 b[k2][n3] W_R3^(n3 k3)
    const int k2 = t / R3, k3 = t % R3;
    v2d acc[4] = {(v2d){0.0, 0.0}, (v2d){0.0, 0.0}, (v2d){0.0, 0.0}, (v2d){0.0, 0.0}};
    const v2d wk = w3[k3];
    v2d w = (v2d){1.0, 0.0};
#pragma unroll
    for (int n3 = 0; n3 < R3; n3++) {
      acc[n3 & 3] += cmul(s_b[k2 * R3 + n3], w);
      w = cmul(w, wk);
    }
    out[(long)row * rs + P::sbase(k1 * R2 + k2) + P::soff(k3)] =
        (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();   // s_a / s_b are refilled by the next (row, k1)
  }
}

// ---- the correlation kernel -------------------------------------------------------
// One workgroup = one unit: BEST_OF_BLOCKS -> (row, block); NONCOHERENT -> row,
// |.|^2 summed over the blocks in registers.  fmap[fid] = {class, m}: the bin's
// spectrum is the class spectrum circularly shifted by m (X_f[k] = X_r[k - m]).
template <class P, int MODE, bool DUMP>
__global__ __launch_bounds__(P::TB) void acq64_corr_kernel(
    const v2d* __restrict__ X, const v2d* __restrict__ F, int rs, int n_blocks,
    const int* __restrict__ group_code, const int* __restrict__ group_freq, int n_bins, int spc,
    gnsscorr_acq_row* __restrict__ stats, double* __restrict__ dump, int dump_block,
    const int* __restrict__ order, const int2* __restrict__ fmap, const v2d* __restrict__ twN,
    int gpr, int nbT, const int* __restrict__ group_rec) {
  constexpr int N = P::N, R1 = P::R1, R3 = P::R3, T = P::T, K3 = P::K3, L = P::L;
  constexpr bool kNC = MODE == GNSSCORR_ACQ_NONCOHERENT;
  // non-coherent: a thread's first kE running sums live in the LDS left over
  // beside the exchange plane for the whole row (the others are parked in the
  // plane between blocks, see start_sums)
  constexpr int kLdsOther = P::LX * 8 + P::LS * 8 + P::NW * 20;
  constexpr int kE0 = kNC ? (kLdsBudget - kLdsOther) / (8 * T) : 0;
  // one s_extra row holds the leftover outputs' sums (pwl) when there are any
  constexpr int kPwlRow = (kNC && L > 0 && kE0 > 0) ? 1 : 0;
  static_assert(!kPwlRow || 2 * P::LT <= T, "leftover sums fit one s_extra row");
  constexpr int kE = kE0 - kPwlRow < K3 * R3 ? kE0 - kPwlRow : K3 * R3;
  __shared__ double lds[P::LX + (kE + kPwlRow) * T];   // the exchange plane, then s_extra
  __shared__ double side[P::LS];
  __shared__ double s_v[P::NW], s_m[P::NW];
  __shared__ int s_k[P::NW];
  static_assert(sizeof(double) * (P::LX + (kE + kPwlRow) * T + P::LS) +
                        (2 * sizeof(double) + sizeof(int)) * P::NW <= (size_t)kLdsBudget,
                "acq64_corr_kernel: static LDS over the gfx950 budget");
  double* const s_extra = lds + P::LX;
  // non-coherent: threadIdx.x is rebuilt inside and after the block loop from the
  // wave's base (uniform: an SGPR) and the lane id, so no per-lane copy of it stays
  // live across the loop (that copy was the kernel's last spill to scratch)
  const int wave_base = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63);
  int t = threadIdx.x;
  const bool act = t < T;
  ACQ64_STAMP(0);
  const int unit = order[blockIdx.x];
  const int rowid = kNC ? unit : unit / n_blocks;
  const int blk0 = kNC ? 0 : unit % n_blocks;
  const int nblk = kNC ? n_blocks : 1;
  // records (gnsscorr_acq_set_records): virtual group gv = rec * gpr + g reads
  // blocks rec * n_blocks .. of the nbT resident blocks per class
  // (gnsscorr_acq_set_group_records: group g searches record group_rec[g] only)
  const int gv = rowid / n_bins, bin = rowid % n_bins;
  // a per-group record outside [0, nbT / n_blocks) is clamped: never a read past the spectra
  const int rec = group_rec ? min(max(group_rec[gv], 0), nbT / n_blocks - 1) : gv / gpr;
  const int g = group_rec ? gv : gv - rec * gpr;
  const int code = group_code[g];
  const int2 fm = fmap[group_freq[g * n_bins + bin]];
  const int m = fm.y;
  const double inv_n2 = 1.0 / ((double)N * (double)N);
  const long fofs0 = (long)code * rs;

  double pw[K3][R3], pwl[2] = {-1.0, -1.0};   // pwl: leftover outputs (P::lvalid)

  for (int i = 0; i < nblk; i++) {
    const int blk = blk0 + i;
    const v2d* Xb = X + ((long)fm.x * nbT + rec * n_blocks + blk) * rs;
    // the code row is the same for every block: keep the compiler from
    // hoisting its loads out of the block loop (they would stay live in
    // registers across the whole transform)
    // (the offset, not the pointer, goes through the asm: an opaque pointer
    // loses its global address space, and the code loads became flat loads,
    // whose completion the waitcnt logic can only wait for all at once)
    long fofs = fofs0;
    asm volatile("" : "+s"(fofs));
    const v2d* Fc = F + fofs;
    // likewise every thread-dependent address: t is opaque per block, so the
    // index arithmetic is redone per block instead of held across it
    int t;
    if constexpr (kNC) {
      t = wave_base + lane_id_opaque();
    } else {
      t = threadIdx.x;
      asm volatile("" : "+v"(t));
    }
    // stage-1 inputs: conj(X[k - m]) * F[k]  (= conj(X * conj(F)), acquisition.sci:116).
    // Slots of groups a thread does not own are left as garbage: fft_core never
    // stores them.
    v2d v1[P::K1][R1];
    if constexpr (P::PFA) {
      constexpr int R2 = P::R2;
      // digits of the shift: X_f[k] = X_r[k - m], negation of m digit-wise
      const int m1 = (m % R1) * P::INV1 % R1, m2 = (m % R2) * P::INV2 % R2,
                m3 = (m % R3) * P::INV3 % R3;
      auto shifted = [&](int g) {
        int n2 = g / R3 - m2, n3 = g % R3 - m3;
        n2 += n2 < 0 ? R2 : 0;
        n3 += n3 < 0 ? R3 : 0;
        return n2 * R3 + n3;
      };
      auto plane = [&](int n1) {
        int a = n1 - m1;
        return (a < 0 ? a + R1 : a) * P::G1;
      };
      if constexpr (P::SYM) {
        // slot 0: group ga; slot 1: gb = -ga, whose code value at plane -n1 is
        // conj(F[ga] at plane n1): one F load serves both
        const int ga0 = P::group1(t, 0), ga = ga0 < 0 ? 0 : ga0;
        const int gb0 = P::group1(t, 1), gb = gb0 < 0 ? ga : gb0;
        const int sa = shifted(ga), sb = shifted(gb);
#pragma unroll
        for (int n1 = 0; n1 < R1; n1++) {
          const int nn = (R1 - n1) % R1;
          const v2d f = Fc[n1 * P::G1 + ga];
          const v2d xa = Xb[plane(n1) + sa], xb = Xb[plane(nn) + sb];
          v1[0][n1] = (v2d){fma(xa.x, f.x, xa.y * f.y), fma(xa.x, f.y, -(xa.y * f.x))};
          v1[1][nn] = (v2d){fma(xb.x, f.x, -(xb.y * f.y)), -fma(xb.x, f.y, xb.y * f.x)};
        }
      } else {
#pragma unroll
        for (int j = 0; j < P::K1; j++) {
          const int g0 = P::group1(t, j), g = g0 < 0 ? 0 : g0;
          const int gs = shifted(g);
#pragma unroll
          for (int n1 = 0; n1 < R1; n1++) {
            const v2d x = Xb[plane(n1) + gs], f = Fc[n1 * P::G1 + g];
            v1[j][n1] = (v2d){fma(x.x, f.x, x.y * f.y), fma(x.x, f.y, -(x.y * f.x))};
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < P::K1; j++) {
        const int g0 = P::group1(t, j), g = g0 < 0 ? 0 : g0;
#pragma unroll
        for (int n1 = 0; n1 < R1; n1++) {
          const int n = n1 * P::G1 + g;
          int s = n - m;
          s += s < 0 ? N : 0;
          const v2d x = Xb[s], f = Fc[n];
          v1[j][n1] = (v2d){fma(x.x, f.x, x.y * f.y), fma(x.x, f.y, -(x.y * f.x))};
        }
      }
    }
    v2d v3[K3][R3], vl[2] = {(v2d){0.0, 0.0}, (v2d){0.0, 0.0}};
    // non-coherent: the running sums are parked in the LDS between blocks
    // (stored after a block's stage 3, when the exchange plane is idle) and
    // come back after this block's stage 1, just before the exchange needs the
    // plane: they are not live across the load phase, whose in-flight X / F
    // loads take the registers (held in registers, they were spilled there).
    auto start_sums = [&]() {
      if constexpr (kNC) {
        // branch-free (a branch here lets the compiler sink stage 1 below the
        // reads, back into the load phase); at i == 0 the plane's content is
        // read but not used
        const bool first = i == 0;
        const int tt = min(t, T - 1);
#pragma unroll
        for (int j = 0; j < K3; j++)
#pragma unroll
          for (int k = 0; k < R3; k++) {
            if (j * R3 + k < kE) continue;   // in s_extra: read just before stage 3
            const double v = lds[(j * R3 + k) * T + tt];
            pw[j][k] = first ? 0.0 : v;
          }
        if constexpr (!kPwlRow) {
          pwl[0] = first ? (P::lvalid(t, 0) ? 0.0 : -1.0) : pwl[0];
          pwl[1] = first ? (P::lvalid(t, 1) ? 0.0 : -1.0) : pwl[1];
        }
        __syncthreads();   // exchange 1 overwrites the parked sums
      }
    };
    // |.|^2 / N^2 (|ifft(Y)|^2 = |fft(conj Y)|^2 / N^2); a prime radix-R3
    // stage is fused with the powers
    constexpr bool kFuse = is_prime(R3);
    fft_core<P, decltype(start_sums), !kFuse, kNC>(lds, side, twN, t, v1, v3, vl,
                                                   start_sums);
    // the first kE running sums are added to in place in s_extra, each read
    // just before its output is formed: they take no registers in stage 3
#pragma unroll
    for (int j = 0; j < K3; j++) {
      auto put_power = [&](int k3, double p) {
        const int f = j * R3 + k3;
        if (kNC && f < kE) {
          if (act) {
            double* const a = s_extra + f * T + t;
            *a = (i == 0 ? 0.0 : *a) + p;
          }
        } else {
          pw[j][k3] = kNC ? pw[j][k3] + p : p;
        }
      };
      if constexpr (kFuse) {
        dft_prime_power<R3>(v3[j], put_power, inv_n2);
      } else {
#pragma unroll
        for (int k3 = 0; k3 < R3; k3++)
          put_power(k3, fma(v3[j][k3].x, v3[j][k3].x, v3[j][k3].y * v3[j][k3].y) * inv_n2);
      }
    }
    if constexpr (L > 0) {
#pragma unroll
      for (int j = 0; j < 2; j++)
        if (P::lvalid(t, j)) {
          const double p = fma(vl[j].x, vl[j].x, vl[j].y * vl[j].y) * inv_n2;
          if constexpr (kPwlRow) {   // in place in the s_extra row after the kE sums
            double* const a = s_extra + kE * T + j * P::LT + t;
            *a = (i == 0 ? 0.0 : *a) + p;
          } else {
            pwl[j] = kNC ? pwl[j] + p : p;
          }
        }
    }
    static_assert(!(DUMP && kNC), "power dumps are coherent-mode only");
    if (DUMP && blk == dump_block && act) {
#pragma unroll
      for (int j = 0; j < K3; j++) {
        int base, step;
        P::out_base(P::group3(t, j), base, step);
        int k = base;
#pragma unroll
        for (int k3 = 0; k3 < R3; k3++) {
          dump[(long)rowid * N + k] = pw[j][k3];
          k += step;
          if (k >= N) k -= N;
        }
      }
      if constexpr (L > 0) {
#pragma unroll
        for (int j = 0; j < 2; j++)
          if (P::lvalid(t, j)) {
            int base, step;
            P::out_base(K3 * T + t % P::L, base, step);
            dump[(long)rowid * N + (base + P::lslot(t, j) * step) % N] = pwl[j];
          }
      }
    }
    if constexpr (kNC) {
      // park the sums (exchange 2's reads ended with a barrier: the plane is idle)
      static_assert(K3 * R3 * T <= N, "parked sums fit the exchange plane");
      if (i + 1 < nblk && act) {
#pragma unroll
        for (int j = 0; j < K3; j++)
#pragma unroll
          for (int k = 0; k < R3; k++) {
            const int f = j * R3 + k;
            if (f >= kE) lds[f * T + t] = pw[j][k];   // f < kE: already in s_extra
          }
      }
    }
  }
  if constexpr (kNC) t = wave_base + lane_id_opaque();
  if constexpr (kE > 0) {
    const int tt = min(t, T - 1);
#pragma unroll
    for (int f = 0; f < kE; f++) pw[f / R3][f % R3] = s_extra[f * T + tt];
  }
  if constexpr (kPwlRow) {
#pragma unroll
    for (int j = 0; j < 2; j++)
      pwl[j] = P::lvalid(t, j) ? s_extra[kE * T + j * P::LT + t] : -1.0;
  }
  // ---- row statistics.  Per stage-3 group, the thread's outputs lie
  // SPACING = N/R3 samples apart, so an exclusion window narrower than that
  // holds at most one of them: a per-group top-2 (max with the first natural
  // index of an exact tie, and the runner-up) gives the largest value outside
  // the window in one pass.  Wider windows (spc > SPACING/2) take an exact
  // second pass over the registers.
  auto wrap_add = [](int k, int d) {   // (k + d) mod N for k, d in [0, N)
    const unsigned u = (unsigned)(k + d);
    return (int)min(u, u - (unsigned)N);
  };
  double a1 = -1.0, a2 = -1.0;
  int ak = INT_MAX;
#pragma unroll
  for (int j = 0; j < K3; j++) {
    int base, step;
    P::out_base(act ? P::group3(t, j) : 0, base, step);
    int k = base;
#pragma unroll
    for (int k3 = 0; k3 < R3; k3++) {
      const double v = pw[j][k3];
      const bool take = v > a1 || (v == a1 && k < ak);
      a2 = fmax(a2, fmin(a1, v));
      ak = take ? k : ak;
      a1 = fmax(a1, v);
      k = wrap_add(k, step);
    }
  }
  if (!act) { a1 = -1.0; a2 = -1.0; ak = INT_MAX; }
  double bv = a1;
  int bk = ak;
  int kl[2] = {INT_MAX, INT_MAX};
  if constexpr (L > 0) {
#pragma unroll
    for (int j = 0; j < 2; j++)
      if (P::lvalid(t, j)) {
        int base, step;
        P::out_base(K3 * T + t % P::L, base, step);
        kl[j] = (base + P::lslot(t, j) * step) % N;
        if (better(pwl[j], kl[j], bv, bk)) { bv = pwl[j]; bk = kl[j]; }
      }
  }
  block_argmax<P::NW>(bv, bk, s_v, s_k, t);
  ACQ64_STAMP(9);
  // second peak: max outside the open circular window (bk - spc, bk + spc)
  auto outside = [&](int k) {
    int d = k - bk;
    d += d < 0 ? N : 0;
    return d >= spc && d <= N - spc;
  };
  double sv = -1.0;
  if (2 * spc - 1 <= P::SPACING) {
    sv = outside(ak) ? a1 : a2;
  } else if (act) {
#pragma unroll
    for (int j = 0; j < K3; j++) {
      int base, step;
      P::out_base(P::group3(t, j), base, step);
      int k = base;
#pragma unroll
      for (int k3 = 0; k3 < R3; k3++) {
        if (outside(k)) sv = fmax(sv, pw[j][k3]);
        k = wrap_add(k, step);
      }
    }
  }
  if constexpr (L > 0) {
#pragma unroll
    for (int j = 0; j < 2; j++)
      if (P::lvalid(t, j) && outside(kl[j])) sv = fmax(sv, pwl[j]);
  }
  sv = block_max0<P::NW>(sv, s_m, t);
  ACQ64_STAMP(10);
  if (t == 0) {
    gnsscorr_acq_row r;
    r.peak = bv;
    r.second = sv;
    r.argmax = bk;
    r.block = kNC ? -1 : blk0;
    stats[(long)rowid * n_blocks + blk0] = r;
  }
}

// Frequencies -> spectrum classes on the fs/N grid: class = canonical residue
// r = f mod fs/N (one forward FFT per class and block); bin f = r + m fs/N
// reads the class spectrum shifted by m.  fmap[i] = {class, m mod N}.
__global__ __launch_bounds__(1024) void acq64_classify_kernel(const double* __restrict__ freqs,
                                                              int n, double delta, int N,
                                                              int2* __restrict__ fmap,
                                                              double* __restrict__ cfreq,
                                                              int* __restrict__ n_classes,
                                                              double* __restrict__ resid,
                                                              int* __restrict__ lead) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) resid[i] = grid_residue(freqs[i], delta);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const double r = resid[i];
    int l = i;
    for (int j = 0; j < i; j++)
      if (resid[j] == r) { l = j; break; }
    lead[i] = l;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int l = lead[i];
    int cls = 0;
    for (int k = 0; k < l; k++) cls += lead[k] == k;
    const double q = rint((freqs[i] - resid[i]) / delta);
    int mN = (fabs(q) < 1e9 ? (int)fmod(q, (double)N) : 0);
    mN += mN < 0 ? N : 0;
    fmap[i] = make_int2(cls, mN);
    if (l == i) cfreq[cls] = resid[i];
  }
  // class count: every thread counts its own entries (one serial thread over
  // the whole table took ~100 us at full-sky sizes, a dependent load per entry)
  __shared__ int s_cnt;
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();
  int mine = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) mine += lead[i] == i;
  atomicAdd(&s_cnt, mine);
  __syncthreads();
  if (threadIdx.x == 0) *n_classes = s_cnt;
}

// ---- launch helpers ---------------------------------------------------------------
template <class P>
int fwd_launch(gnsscorr_acq_ctx* c, const v2d* in, const int* n_cls_dev, int per_cls,
               int n_rows, v2d* out) {
  if constexpr (P::PFA) {
    // two launches spread over the whole GPU (a config-2 search has only 4
    // rows: one workgroup per row would leave 252 CUs idle): stage 1 in place,
    // then the 16 independent 1023-point (33 x 31) transforms of every row
    v2d* io = const_cast<v2d*>(in);
    // n_rows is an upper bound when the class count is on the device (a
    // full-sky GLONASS part: 574 frequencies x 10 blocks for 2 classes x 10):
    // capped grids, grid-stride kernels (92 k mostly-empty workgroups cost
    // ~190 us of launch alone)
    const long groups = (long)n_rows * P::G1;
    const long g1 = (groups + 255) / 256, g23 = (long)n_rows * P::R1;
    hipLaunchKernelGGL((acq64_fwd1_kernel<P>), dim3((unsigned)(g1 < 4096 ? g1 : 4096)), dim3(256),
                       0, c->stream, io, n_cls_dev, per_cls, n_rows);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL((acq64_fwd23_kernel<P>), dim3((unsigned)(g23 < 2048 ? g23 : 2048)),
                       dim3(kFwd23Threads), 0, c->stream, (const v2d*)io, n_cls_dev, per_cls,
                       n_rows, out, c->rs64);
  } else {
    hipLaunchKernelGGL((acq64_fwd_kernel<P>), dim3(n_rows < 512 ? n_rows : 512), dim3(P::TB), 0,
                       c->stream, in,
                       n_cls_dev, per_cls, n_rows, out, c->rs64, (const v2d*)c->d_twN);
  }
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

template <class P>
int corr_launch(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_units, int n_bins,
                const int32_t* d_gcode, const int32_t* d_gfreq, int spc, double* d_dump,
                int dump_block, int gpr) {
  const int nbT = n_blocks * c->spec_recs;

#define ACQ64_LAUNCH(M, D)                                                                  \
  hipLaunchKernelGGL((acq64_corr_kernel<P, M, D>), dim3(n_units), dim3(P::TB), 0, c->stream, \
                     (const v2d*)c->d_X64, (const v2d*)c->d_F64, c->rs64, n_blocks, d_gcode,   \
                     d_gfreq, n_bins, spc, c->d_stats, d_dump, dump_block, c->d_order,         \
                     c->d_fmap64, (const v2d*)c->d_twN, gpr, nbT, c->d_group_rec)
  if (d_dump)
    ACQ64_LAUNCH(GNSSCORR_ACQ_BEST_OF_BLOCKS, true);
  else if (mode == GNSSCORR_ACQ_NONCOHERENT)
    ACQ64_LAUNCH(GNSSCORR_ACQ_NONCOHERENT, false);
  else
    ACQ64_LAUNCH(GNSSCORR_ACQ_BEST_OF_BLOCKS, false);
#undef ACQ64_LAUNCH
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

}  // namespace

// ==================================================================================
// Generic N (any other samplesPerCode, e.g. acquisition.sci at fs = 5 or 38.192 MHz):
// the same fp64 pipeline with every length-N DFT done by Bluestein's chirp-z
// identity  X_k = c_k sum_n (a_n c_n) conj(c_{k-n}),  c_n = exp(-i pi n^2 / N),
// i.e. a cyclic convolution of length M = 2^q >= 2N - 1 (radix-16 Stockham
// passes in global memory, the last one radix 2, 4 or 8 when q is not a
// multiple of 4).  A fallback for sizes without a compiled plan: correct to
// fp64 rounding, not tuned.
// ==================================================================================
namespace {

constexpr int kGThreads = 256;

// one radix-R Stockham pass (autosort), forward: Ns = product of the earlier
// passes' radices
template <int R>
__global__ __launch_bounds__(kGThreads) void g_fft_pass(const v2d* __restrict__ in,
                                                        v2d* __restrict__ out, int M, int Ns,
                                                        const v2d* __restrict__ twM) {
  const int j = blockIdx.x * kGThreads + threadIdx.x;   // < M / R
  const long row = (long)blockIdx.y * M;
  if (j >= M / R) return;
  const int k = j & (Ns - 1);
  const int tstep = k * (M / (R * Ns));                   // twiddle W_M^(r * tstep)
  v2d v[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const v2d x = in[row + j + r * (M / R)];
    v[r] = r == 0 ? x : cmul(x, twM[(r * tstep) & (M - 1)]);
  }
  dft<R>(v);
  const int d = (j / Ns) * Ns * R + k;
#pragma unroll
  for (int r = 0; r < R; r++) out[row + d + r * Ns] = v[r];
}

// A[row] = (a_n c_n | 0...) from natural rows a (stride src_rs)
__global__ __launch_bounds__(kGThreads) void g_pre_kernel(const v2d* __restrict__ a, int src_rs,
                                                          const v2d* __restrict__ chirp, int N,
                                                          int M, v2d* __restrict__ A) {
  const int n = blockIdx.x * kGThreads + threadIdx.x;
  if (n >= M) return;
  const long r = blockIdx.y;
  A[r * M + n] = n < N ? cmul(a[r * src_rs + n], chirp[n]) : (v2d){0.0, 0.0};
}

// correlation rows of a chunk: Y_k = conj(X_cls,blk[k - m]) F_code[k] (as acq64_corr_kernel),
// times c_k, zero padded.  unit = u0 + blockIdx.y; block `blk` of it (-1: the unit's own).
__global__ __launch_bounds__(kGThreads) void g_corr_pre_kernel(
    const v2d* __restrict__ X, const v2d* __restrict__ F, int rs, int n_blocks, int nc_blk,
    const int* __restrict__ group_code, const int* __restrict__ group_freq, int n_bins,
    const int2* __restrict__ fmap, int u0, const v2d* __restrict__ chirp, int N, int M,
    v2d* __restrict__ A) {
  const int n = blockIdx.x * kGThreads + threadIdx.x;
  if (n >= M) return;
  const int unit = u0 + blockIdx.y;
  const int rowid = nc_blk >= 0 ? unit : unit / n_blocks;
  const int blk = nc_blk >= 0 ? nc_blk : unit % n_blocks;
  const int g = rowid / n_bins, bin = rowid % n_bins;
  v2d y = (v2d){0.0, 0.0};
  if (n < N) {
    const int2 fm = fmap[group_freq[g * n_bins + bin]];
    int s = n - fm.y;
    s += s < 0 ? N : 0;
    const v2d x = X[((long)fm.x * n_blocks + blk) * rs + s];
    const v2d f = F[(long)group_code[g] * rs + n];
    y = cmul((v2d){fma(x.x, f.x, x.y * f.y), fma(x.x, f.y, -(x.y * f.x))}, chirp[n]);
  }
  A[(long)blockIdx.y * M + n] = y;
}

// B = conj(A * Vf)   (IFFT_M(Z) = conj(FFT_M(conj Z)) / M)
__global__ __launch_bounds__(kGThreads) void g_mulv_kernel(const v2d* __restrict__ A,
                                                           const v2d* __restrict__ vf, int M,
                                                           v2d* __restrict__ B) {
  const int n = blockIdx.x * kGThreads + threadIdx.x;
  if (n >= M) return;
  const long i = (long)blockIdx.y * M + n;
  const v2d z = cmul(A[i], vf[n]);
  B[i] = (v2d){z.x, -z.y};
}

// spectra: out[k] = c_k conj(D_k) / M
__global__ __launch_bounds__(kGThreads) void g_post_kernel(const v2d* __restrict__ D,
                                                           const v2d* __restrict__ chirp, int N,
                                                           int M, v2d* __restrict__ out, int rs) {
  const int k = blockIdx.x * kGThreads + threadIdx.x;
  if (k >= N) return;
  const v2d d = D[(long)blockIdx.y * M + k];
  const double inv = 1.0 / (double)M;
  out[(long)blockIdx.y * rs + k] = cmul((v2d){d.x * inv, -d.y * inv}, chirp[k]);
}

// powers |DFT_N(Y)|^2 / N^2 = |D_k|^2 / (M N)^2, stored or added
__global__ __launch_bounds__(kGThreads) void g_power_kernel(const v2d* __restrict__ D, int N,
                                                            int M, int acc,
                                                            double* __restrict__ pw) {
  const int k = blockIdx.x * kGThreads + threadIdx.x;
  if (k >= N) return;
  const v2d d = D[(long)blockIdx.y * M + k];
  const double sc = 1.0 / ((double)M * (double)N);
  const double p = fma(d.x * sc, d.x * sc, (d.y * sc) * (d.y * sc));
  double* o = pw + (long)blockIdx.y * N + k;
  *o = acc ? *o + p : p;
}

// row statistics of a power row (acq64_corr_kernel's: first natural index of
// the maximum, max outside the open circular window (argmax - spc, argmax + spc))
__global__ __launch_bounds__(kGThreads) void g_stats_kernel(const double* __restrict__ pw, int N,
                                                            int u0, int n_blocks, int nc, int spc,
                                                            gnsscorr_acq_row* __restrict__ stats,
                                                            double* __restrict__ dump,
                                                            int dump_block) {
  __shared__ double s_v[kGThreads / 64], s_m[kGThreads / 64];
  __shared__ int s_k[kGThreads / 64];
  const int unit = u0 + blockIdx.x;
  const double* row = pw + (long)blockIdx.x * N;
  const int rowid = nc ? unit : unit / n_blocks;
  const int blk0 = nc ? 0 : unit % n_blocks;
  double bv = -1.0;
  int bk = INT_MAX;
  for (int k = threadIdx.x; k < N; k += kGThreads)
    if (row[k] > bv) { bv = row[k]; bk = k; }     // first index within the thread's stride
  block_argmax<kGThreads / 64>(bv, bk, s_v, s_k);
  double sv = -1.0;
  for (int k = threadIdx.x; k < N; k += kGThreads) {
    int d = k - bk;
    d += d < 0 ? N : 0;
    if (d >= spc && d <= N - spc) sv = fmax(sv, row[k]);
  }
  sv = block_max0<kGThreads / 64>(sv, s_m);
  if (dump && !nc && blk0 == dump_block)
    for (int k = threadIdx.x; k < N; k += kGThreads) dump[(long)rowid * N + k] = row[k];
  if (threadIdx.x == 0) {
    gnsscorr_acq_row r;
    r.peak = bv;
    r.second = sv;
    r.argmax = bk;
    r.block = nc ? -1 : blk0;
    stats[(long)rowid * n_blocks + blk0] = r;
  }
}

// One-pass row statistics (the generic path's default): 1024 threads, thread t
// scans k = t, t + 1024, ...  Its elements lie 1024 samples apart (fewer across the
// wrap, stats1_exact), so the open window (argmax - spc, argmax + spc) holds at most
// one of them when stats1_exact: the thread's runner-up stands in for its maximum when
// that maximum is
// inside the window (acq64_corr_kernel's per-thread top-2).  Same results as
// g_stats_kernel's two passes; one read of the row.
constexpr int kStatsThreads = 1024;
// g_stats1_kernel is exact when no thread holds two samples inside one open window
// of 2 spc - 1 positions.  A thread's samples are kStatsThreads apart, except across
// the wrap: thread t's last sample t + kStatsThreads q and its first lie N - kStatsThreads q
// apart, smallest (r = N - kStatsThreads floor((N - 1) / kStatsThreads)) for the
// threads with the most samples (304 at N = 38192, 16 at N = 16400).
static inline bool stats1_exact(int N, int spc) {
  const int r = N <= kStatsThreads ? kStatsThreads : N - kStatsThreads * ((N - 1) / kStatsThreads);
  return 2 * spc - 1 <= (r < kStatsThreads ? r : kStatsThreads);
}
__global__ __launch_bounds__(kStatsThreads) void g_stats1_kernel(
    const double* __restrict__ pw, int N, int u0, int n_blocks, int nc, int spc,
    gnsscorr_acq_row* __restrict__ stats, double* __restrict__ dump, int dump_block) {
  __shared__ double s_v[kStatsThreads / 64], s_m[kStatsThreads / 64];
  __shared__ int s_k[kStatsThreads / 64];
  const int unit = u0 + blockIdx.x;
  const double* row = pw + (long)blockIdx.x * N;
  const int rowid = nc ? unit : unit / n_blocks;
  const int blk0 = nc ? 0 : unit % n_blocks;
  double a1 = -1.0, a2 = -1.0;
  int ak = INT_MAX;
  for (int k = threadIdx.x; k < N; k += kStatsThreads) {
    const double v = row[k];
    a2 = v > a1 ? a1 : fmax(a2, v);
    ak = v > a1 ? k : ak;       // strict: the first index of the thread's maximum
    a1 = fmax(a1, v);
  }
  double bv = a1;
  int bk = ak;
  block_argmax<kStatsThreads / 64>(bv, bk, s_v, s_k);
  int d = ak == INT_MAX ? 0 : ak - bk;
  d += d < 0 ? N : 0;
  double sv = (ak != INT_MAX && d >= spc && d <= N - spc) ? a1 : a2;
  sv = block_max0<kStatsThreads / 64>(sv, s_m);
  if (dump && !nc && blk0 == dump_block)
    for (int k = threadIdx.x; k < N; k += kStatsThreads) dump[(long)rowid * N + k] = row[k];
  if (threadIdx.x == 0) {
    gnsscorr_acq_row r;
    r.peak = bv;
    r.second = sv;
    r.argmax = bk;
    r.block = nc ? -1 : blk0;
    stats[(long)rowid * n_blocks + blk0] = r;
  }
}

// wipe-off rows in natural order (acq64_wipe_kernel with a runtime N)
__global__ __launch_bounds__(256) void g_wipe_kernel(const int8_t* __restrict__ src, int iq,
                                                     int n_blocks, int coh,
                                                     const double* __restrict__ cfreq,
                                                     const int* __restrict__ n_cls_dev, double ts,
                                                     int N, v2d* __restrict__ out) {
  const long total = (long)(*n_cls_dev) * n_blocks * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int row = (int)(i / N), n = (int)(i % N);
    const int cls = row / n_blocks, blk = row % n_blocks;
    const double f = cfreq[cls];
    const bool cplx = iq & GNSSCORR_IF_IQ, pk = iq & GNSSCORR_IF_PACKED2;
    const int ne = cplx ? 2 : 1;
    const long e0 = (long)blk * coh * N * ne;
    double re = 0.0, im = 0.0;
    for (int p = 0; p < coh; p++) {
      const long m = n + (long)p * N;
      const double I = (double)if_elem(src, e0 + ne * m, pk);
      const double Q = cplx ? (double)if_elem(src, e0 + 2 * m + 1, pk) : 0.0;
      const double th = f * ((((double)m * 2.0) * M_PI) * ts);
      double sn, cs;
      sincos(th, &sn, &cs);
      re += I * cs - Q * sn;
      im += I * sn + Q * cs;
    }
    out[(long)row * N + n] = (v2d){re, im};
  }
}

__global__ __launch_bounds__(256) void g_codes_kernel(const int8_t* __restrict__ codes, long n,
                                                      v2d* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (v2d){(double)codes[i], 0.0};
}

// FFT_M of `rows` rows in place in A (B is the ping-pong buffer); result in *res
int g_fft(gnsscorr_acq_ctx* c, v2d* A, v2d* B, int rows, v2d** res) {
  const int M = c->gM;
  v2d *in = A, *out = B;
  int Ns = 1;
  while (Ns < M) {
    const int R = M / Ns >= 16 ? 16 : M / Ns;   // radix-16 passes, then one of 2, 4 or 8
    const dim3 grid((M / R + kGThreads - 1) / kGThreads, rows);
    const v2d* tw = (const v2d*)c->d_twM;
    if (R == 16)
      hipLaunchKernelGGL(g_fft_pass<16>, grid, dim3(kGThreads), 0, c->stream, in, out, M, Ns, tw);
    else if (R == 8)
      hipLaunchKernelGGL(g_fft_pass<8>, grid, dim3(kGThreads), 0, c->stream, in, out, M, Ns, tw);
    else if (R == 4)
      hipLaunchKernelGGL(g_fft_pass<4>, grid, dim3(kGThreads), 0, c->stream, in, out, M, Ns, tw);
    else
      hipLaunchKernelGGL(g_fft_pass<2>, grid, dim3(kGThreads), 0, c->stream, in, out, M, Ns, tw);
    HIP_TRY(hipGetLastError());
    Ns *= R;
    v2d* t = in;
    in = out;
    out = t;
  }
  *res = in;
  return GNSSCORR_OK;
}

// DFT_N of `rows` natural rows a (stride src_rs) -> out (stride rs), via chunks
int g_dft_rows(gnsscorr_acq_ctx* c, const v2d* a, int src_rs, int rows, v2d* out, int rs) {
  const int N = c->cfg.n_samples, M = c->gM;
  for (int r0 = 0; r0 < rows; r0 += c->g_chunk) {
    const int nr = rows - r0 < c->g_chunk ? rows - r0 : c->g_chunk;
    v2d *A = (v2d*)c->d_gA, *B = (v2d*)c->d_gB, *D;
    hipLaunchKernelGGL(g_pre_kernel, dim3((M + kGThreads - 1) / kGThreads, nr), dim3(kGThreads),
                       0, c->stream, a + (long)r0 * src_rs, src_rs, (const v2d*)c->d_chirp, N, M,
                       A);
    HIP_TRY(hipGetLastError());
    int rc = g_fft(c, A, B, nr, &D);
    if (rc) return rc;
    v2d* E = D == A ? B : A;
    hipLaunchKernelGGL(g_mulv_kernel, dim3((M + kGThreads - 1) / kGThreads, nr), dim3(kGThreads),
                       0, c->stream, D, (const v2d*)c->d_vf, M, E);
    HIP_TRY(hipGetLastError());
    rc = g_fft(c, E, D, nr, &D);
    if (rc) return rc;
    hipLaunchKernelGGL(g_post_kernel, dim3((N + kGThreads - 1) / kGThreads, nr), dim3(kGThreads),
                       0, c->stream, D, (const v2d*)c->d_chirp, N, M, out + (long)r0 * rs, rs);
    HIP_TRY(hipGetLastError());
  }
  return GNSSCORR_OK;
}

// rows per chunk of the generic engine: at most what one call of this context
// can run in one go (codes x frequencies x blocks covers the code spectra, the IF
// class spectra and a search's units), so small contexts keep small work buffers
// (ADVICE r5); 1 .. 4096
int chunk_cap(const gnsscorr_acq_ctx* c, int rows) {
  const long most = (long)c->cfg.max_codes * c->cfg.max_freqs * c->cfg.max_blocks;
  if (rows > most) rows = (int)(most < 4096 ? most : 4096);
  if (rows > 4096) rows = 4096;
  return rows < 1 ? 1 : rows;
}

int g_init(gnsscorr_acq_ctx* c) {
  const long N = c->cfg.n_samples;
  int M = 16, P = 0;   // P: passes (radix 16, the last possibly 2 / 4 / 8)
  while (M < 2 * N - 1) M *= 2;
  for (int m = 1; m < M; m *= 16) P++;
  c->gM = M;
  c->gP = P;
  // chunk: ~64 MiB per work buffer
  c->g_chunk = chunk_cap(c, (int)((64L << 20) / ((long)M * 16)));
  HIP_TRY(hipMalloc(&c->d_chirp, sizeof(double2) * N));
  HIP_TRY(hipMalloc(&c->d_vf, sizeof(double2) * M));
  HIP_TRY(hipMalloc(&c->d_twM, sizeof(double2) * M));
  HIP_TRY(hipMalloc(&c->d_gA, sizeof(double2) * (size_t)M * c->g_chunk));
  HIP_TRY(hipMalloc(&c->d_gB, sizeof(double2) * (size_t)M * c->g_chunk));
  HIP_TRY(hipMalloc(&c->d_gpw, sizeof(double) * (size_t)N * c->g_chunk));
  double2* h = (double2*)malloc(sizeof(double2) * M);
  if (!h) return GNSSCORR_ENOMEM;
  // chirp: exact argument reduction n^2 mod 2N
  for (long n = 0; n < N; n++) {
    const long q = (n * n) % (2 * N);
    const double a = -M_PI * ((double)q / (double)N);
    h[n] = make_double2(cos(a), sin(a));
  }
  hipError_t e = hipMemcpy(c->d_chirp, h, sizeof(double2) * N, hipMemcpyHostToDevice);
  // W_M^t with the angle reduced to the first octant by symmetry
  for (long t = 0; e == hipSuccess && t < M; t++) {
    const double a = -2.0 * M_PI * ((double)t / (double)M);
    h[t] = make_double2(cos(a), sin(a));
  }
  if (e == hipSuccess) e = hipMemcpy(c->d_twM, h, sizeof(double2) * M, hipMemcpyHostToDevice);
  // two-sided conjugate chirp v_m = conj(c_|m|), wrapped to M
  for (long m = 0; m < M; m++) h[m] = make_double2(0.0, 0.0);
  for (long m = 0; m < N; m++) {
    const long q = (m * m) % (2 * N);
    const double a = M_PI * ((double)q / (double)N);
    h[m] = make_double2(cos(a), sin(a));
    if (m > 0) h[M - m] = h[m];
  }
  if (e == hipSuccess) e = hipMemcpy(c->d_gA, h, sizeof(double2) * M, hipMemcpyHostToDevice);
  free(h);
  HIP_TRY(e);
  v2d* D;
  int rc = g_fft(c, (v2d*)c->d_gA, (v2d*)c->d_gB, 1, &D);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_vf, D, sizeof(double2) * M, hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

int mx_dft_rows(gnsscorr_acq_ctx* c, const v2d* a, int src_rs, int rows, v2d* out, int rs);
int mx_correlate(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_groups, int n_bins,
                 const int32_t* d_gcode, const int32_t* d_gfreq, int spc, double* d_dump,
                 int dump_block);

// DFT_N of natural rows: the mixed-radix plan where N has one, else Bluestein
int gen_dft_rows(gnsscorr_acq_ctx* c, const v2d* a, int src_rs, int rows, v2d* out, int rs) {
  return c->mix_nr ? mx_dft_rows(c, a, src_rs, rows, out, rs)
                   : g_dft_rows(c, a, src_rs, rows, out, rs);
}

int g_set_codes(gnsscorr_acq_ctx* c, const int8_t* d_codes, int n_codes) {
  const long n = (long)n_codes * c->cfg.n_samples;
  hipLaunchKernelGGL(g_codes_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, d_codes, n,
                     (v2d*)c->d_in64);
  HIP_TRY(hipGetLastError());
  return gen_dft_rows(c, (const v2d*)c->d_in64, c->cfg.n_samples, n_codes, (v2d*)c->d_F64, c->rs64);
}

int g_spectra(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq, int n_blocks, int n_freqs,
              const double* d_freqs) {
  const int N = c->cfg.n_samples;
  hipLaunchKernelGGL(acq64_classify_kernel, dim3(1), dim3(1024), 0, c->stream, d_freqs, n_freqs,
                     c->cfg.samp_rate / N, N, c->d_fmap64, c->d_cfreq, c->d_nclass, c->d_resid,
                     c->d_lead64);
  HIP_TRY(hipGetLastError());
  const int rows = n_freqs * n_blocks;   // upper bound: classes <= frequencies
  const long work = (long)rows * N;
  const int grid = (int)((work + 255) / 256 < 2048 ? (work + 255) / 256 : 2048);
  hipLaunchKernelGGL(g_wipe_kernel, dim3(grid), dim3(256), 0, c->stream, d_if, iq, n_blocks,
                     c->coh, (const double*)c->d_cfreq, (const int*)c->d_nclass,
                     1.0 / c->cfg.samp_rate, N, (v2d*)c->d_in64);
  HIP_TRY(hipGetLastError());
  // transform only the class rows (the count is on the device: one small read
  // back; this generic path is synchronous here anyway)
  int n_cls = 0;
  HIP_TRY(hipMemcpyAsync(&n_cls, c->d_nclass, sizeof(int), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return gen_dft_rows(c, (const v2d*)c->d_in64, N, n_cls * n_blocks, (v2d*)c->d_X64, c->rs64);
}

int g_correlate(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_groups, int n_bins,
                const int32_t* d_gcode, const int32_t* d_gfreq, int spc, double* d_dump,
                int dump_block) {
  if (c->mix_nr)
    return mx_correlate(c, n_blocks, mode, n_groups, n_bins, d_gcode, d_gfreq, spc, d_dump,
                        dump_block);
  const int N = c->cfg.n_samples, M = c->gM;
  const bool nc = mode == GNSSCORR_ACQ_NONCOHERENT;
  const int n_units = n_groups * n_bins * (nc ? 1 : n_blocks);
  for (int u0 = 0; u0 < n_units; u0 += c->g_chunk) {
    const int nu = n_units - u0 < c->g_chunk ? n_units - u0 : c->g_chunk;
    for (int b = 0; b < (nc ? n_blocks : 1); b++) {
      v2d *A = (v2d*)c->d_gA, *B = (v2d*)c->d_gB, *D;
      hipLaunchKernelGGL(g_corr_pre_kernel, dim3((M + kGThreads - 1) / kGThreads, nu),
                         dim3(kGThreads), 0, c->stream, (const v2d*)c->d_X64,
                         (const v2d*)c->d_F64, c->rs64, n_blocks, nc ? b : -1, d_gcode, d_gfreq,
                         n_bins, (const int2*)c->d_fmap64, u0, (const v2d*)c->d_chirp, N, M, A);
      HIP_TRY(hipGetLastError());
      int rc = g_fft(c, A, B, nu, &D);
      if (rc) return rc;
      v2d* E = D == A ? B : A;
      hipLaunchKernelGGL(g_mulv_kernel, dim3((M + kGThreads - 1) / kGThreads, nu),
                         dim3(kGThreads), 0, c->stream, D, (const v2d*)c->d_vf, M, E);
      HIP_TRY(hipGetLastError());
      rc = g_fft(c, E, D, nu, &D);
      if (rc) return rc;
      hipLaunchKernelGGL(g_power_kernel, dim3((N + kGThreads - 1) / kGThreads, nu),
                         dim3(kGThreads), 0, c->stream, D, N, M, b > 0, c->d_gpw);
      HIP_TRY(hipGetLastError());
    }
    if (stats1_exact(N, spc))
      hipLaunchKernelGGL(g_stats1_kernel, dim3(nu), dim3(kStatsThreads), 0, c->stream,
                         (const double*)c->d_gpw, N, u0, n_blocks, (int)nc, spc, c->d_stats,
                         d_dump, dump_block);
    else
      hipLaunchKernelGGL(g_stats_kernel, dim3(nu), dim3(kGThreads), 0, c->stream,
                         (const double*)c->d_gpw, N, u0, n_blocks, (int)nc, spc, c->d_stats,
                         d_dump, dump_block);
    HIP_TRY(hipGetLastError());
  }
  return GNSSCORR_OK;
}

// ---------------------------------------------------------------------------------
// Mixed-radix Stockham FFT of length N (the generic path's default since round 5):
// N = R_1 ... R_P, every R_i a radix the kernels are compiled for (mix_factor).
// Pass i (Ns = R_1 ... R_{i-1}) reads elements j + r N/R_i (r < R_i) of a row,
// multiplies element r by W_{Ns R}^{r k} (k = j mod Ns; = W_N^{r k N/(Ns R)}, the
// table d_twN), runs a radix-R DFT in registers (dft<R>) and writes positions
// (j / Ns) Ns R + k + r Ns: autosort, natural order out, no bit reversal.
// Against Bluestein (two FFTs of length M = 2^q >= 2N - 1 per DFT plus the chirp
// passes, ~60 N x 16 B of row traffic per correlation row at N = 38 192) a
// correlation row moves ~5.5 N x 16 B: the product conj(X[k - m]) F[k] is formed
// inside the first pass and |.|^2 / N^2 inside the last (added over the blocks of a
// non-coherent search), so no pre / post passes run (acquisition.sci:107-132).
// ---------------------------------------------------------------------------------
constexpr int kMixThreads = 128;
#ifndef MX_WAVES
#define MX_WAVES 3
#endif

struct MixCorr {
  const v2d* X;
  const v2d* F;
  int rs, n_blocks, nc_blk, n_bins, u0;
  const int* group_code;
  const int* group_freq;
  const int2* fmap;
  // records (gnsscorr_acq_set_records): virtual group g = rec * n_groups + g0 searches
  // group g0 on record rec, whose blocks are rec * n_blocks ... of the spectra's nbT
  int n_groups = 1 << 30, nbT = 0;
};

// a correlation unit's class spectrum row and code spectrum row (MODE 1 of the passes)
__device__ __forceinline__ void mix_unit_rows(const MixCorr& cp, int unit, const v2d*& Xr,
                                              const v2d*& Fr, int& shift) {
  const int rowid = cp.nc_blk >= 0 ? unit : unit / cp.n_blocks;
  const int blk = cp.nc_blk >= 0 ? cp.nc_blk : unit % cp.n_blocks;
  const int g = rowid / cp.n_bins, bin = rowid % cp.n_bins;
  const int rec = g / cp.n_groups, g0 = g - rec * cp.n_groups;
  const int2 fm = cp.fmap[cp.group_freq[g0 * cp.n_bins + bin]];
  Xr = cp.X + ((long)fm.x * cp.nbT + rec * cp.n_blocks + blk) * cp.rs;
  Fr = cp.F + (long)cp.group_code[g0] * cp.rs;
  shift = fm.y;
}

// MODE 0: rows in (stride in_rs) -> rows out (stride out_rs)
// MODE 1: first pass of a correlation chunk: the input is y[n] = conj(X[n - m]) F[n] of
//         unit u0 + row (its bin's class spectrum shifted by m, acquisition.sci:116)
// MODE 2: last pass of a correlation chunk: |.|^2 / N^2 into pw (added when acc)
// occupancy: a pass is latency bound (strided row loads, one butterfly per thread),
// so the register allocator is held to 3 waves per SIMD up to radix 16 (the fused
// first pass otherwise keeps all 2R complex loads in flight: 244 VGPRs, 2 waves;
// at 4 waves radix 16 spills)
template <int R>
constexpr int mx_waves() { return R <= 16 ? MX_WAVES : 2; }
template <int R, int MODE>
__global__ __launch_bounds__(kMixThreads, mx_waves<R>()) void mx_pass(const v2d* __restrict__ in, int in_rs,
                                                       v2d* __restrict__ out, int out_rs, int N,
                                                       int Ns, const v2d* __restrict__ tw,
                                                       MixCorr cp, double* __restrict__ pw,
                                                       int acc) {
  const int j = blockIdx.x * kMixThreads + threadIdx.x;   // < N / R
  if (j >= N / R) return;
  const long row = blockIdx.y;
  const int NR = N / R;
  v2d v[R];
  if constexpr (MODE == 1) {
    const v2d *Xr, *Fr;
    int shift;
    mix_unit_rows(cp, cp.u0 + (int)row, Xr, Fr, shift);
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int n = j + r * NR;
      int s = n - shift;
      s += s < 0 ? N : 0;
      const v2d x = Xr[s], f = Fr[n];
      v[r] = (v2d){fma(x.x, f.x, x.y * f.y), fma(x.x, f.y, -(x.y * f.x))};
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = in[row * in_rs + j + r * NR];
  }
  const int k = j % Ns;
  const int ts = k * (N / (Ns * R));   // r ts < N
#pragma unroll
  for (int r = 1; r < R; r++) v[r] = cmul(v[r], tw[r * ts]);
  dft<R>(v);
  const int d = (j / Ns) * Ns * R + k;
  if constexpr (MODE == 2) {
    const double sc = 1.0 / ((double)N * (double)N);
    double* o = pw + row * N + d;
#pragma unroll
    for (int r = 0; r < R; r++) {
      const double q = fma(v[r].x, v[r].x, v[r].y * v[r].y) * sc;
      o[r * Ns] = acc ? o[r * Ns] + q : q;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; r++) out[row * out_rs + d + r * Ns] = v[r];
  }
}

// the radices mx_pass is compiled for, largest first within a power of two
#define MIX_RADICES(X) X(16) X(8) X(4) X(2) X(3) X(5) X(7) X(11) X(13) X(17) X(19) X(23) X(29) X(31)

// N -> radices (powers of two as 16s, then one 8 / 4 / 2; odd primes); 0 when a
// prime factor above 31 remains (Bluestein).  38192 -> 7, 16, 31, 11.
int mix_factor(int N, int* r) {
  int n = 0, m = N;
  while (m % 16 == 0 && n < 24) { r[n++] = 16; m /= 16; }
  if (m % 8 == 0) { r[n++] = 8; m /= 8; }
  else if (m % 4 == 0) { r[n++] = 4; m /= 4; }
  else if (m % 2 == 0) { r[n++] = 2; m /= 2; }
  const int odd[] = {3, 5, 7, 11, 13, 17, 19, 23, 29, 31};
  for (int p : odd)
    while (m % p == 0 && n < 24) { r[n++] = p; m /= p; }
  if (m != 1 || n < 2) return 0;
  // the fused passes take the smallest radices (fewest registers): the first (the
  // correlation product, 2R loads) the smallest, the last (|.|^2) the next one
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++)
      if (r[b] < r[a]) { const int t = r[a]; r[a] = r[b]; r[b] = t; }
  const int second = r[1];
  for (int a = 1; a + 1 < n; a++) r[a] = r[a + 1];
  r[n - 1] = second;
  return n;
}

template <int MODE>
int mx_launch(gnsscorr_acq_ctx* c, int R, const v2d* in, int in_rs, v2d* out, int out_rs, int rows,
              int Ns, const MixCorr& cp, double* pw, int acc) {
  const int N = c->cfg.n_samples;
  const dim3 grid((N / R + kMixThreads - 1) / kMixThreads, rows);
  const v2d* tw = (const v2d*)c->d_twN;
  switch (R) {
#define MIX_CASE(RR)                                                                           \
  case RR:                                                                                     \
    hipLaunchKernelGGL((mx_pass<RR, MODE>), grid, dim3(kMixThreads), 0, c->stream, in, in_rs, \
                       out, out_rs, N, Ns, tw, cp, pw, acc);                                   \
    break;
    MIX_RADICES(MIX_CASE)
#undef MIX_CASE
    default:
      gnsscorr_set_error("acq64 mixed radix: no kernel for radix %d", R);
      return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

// ---------------------------------------------------------------------------------
// Four-step plan (round 5): N = N1 N2 with N1 = A B and N2 = C D, each a pair of
// compiled radices.  X[k1 + N1 k2] = sum_n2 W_N2^(n2 k2) W_N^(n2 k1) sum_n1
// W_N1^(n1 k1) x[N2 n1 + n2].  m4_cols2 runs the N1-point DFTs of a tile of kM4T2
// columns n2 in LDS (A-point DFTs, twiddle W_N1^(q u), B-point DFTs: the standard
// two-factor split), multiplies by W_N^(n2 k1) and writes Y[k1 N2 + n2]; m4_rows
// (m4_rows2) runs the N2-point DFTs of kR2 rows k1 the same way and writes X[k1 + N1 k2].
// Two passes over the rows instead of the four of the mixed-radix plan at
// N = 38 192 = 112 x 341; the correlation product is formed in the first, |.|^2 /
// N^2 in the second (acquisition.sci:107-132), as in mx_pass.
// ---------------------------------------------------------------------------------
#ifndef M4_CT
#define M4_CT 128   // m4_cols2 threads
#endif
#ifndef M4_T2
#define M4_T2 16    // m4_cols2: columns n2 per workgroup
#endif
#ifndef M4_RT
#define M4_RT 64    // m4_rows2 threads
#endif
#ifndef M4_COLS2_PLANE
#define M4_COLS2_PLANE 1   // m4_cols2: exchange through one fp64 plane at a time (0: complex)
#endif
#ifndef M4_COLS2_WPE
#define M4_COLS2_WPE 4     // m4_cols2: waves per SIMD the allocator is held to (0: free)
#endif
#if M4_COLS2_WPE
#define M4_COLS2_ATTR __attribute__((amdgpu_waves_per_eu(M4_COLS2_WPE)))
#else
#define M4_COLS2_ATTR
#endif
constexpr int kM4ColThreads = M4_CT, kM4T2 = M4_T2, kM4RowThreads = M4_RT;
// The intermediate rows Y[k1][n2] are stored at a pitch of N2 rounded up to whole
// m4_cols2 tiles (kM4T2 columns = 256 B): every tile writes whole, aligned 128-byte
// lines that no other workgroup touches (at the natural pitch N2 = 341 a tile's
// 256-byte runs straddled three lines shared with the neighbouring tiles, which run
// on other XCDs)
__host__ __device__ constexpr int m4_pitch(int n2) { return (n2 + kM4T2 - 1) / kM4T2 * kM4T2; }


// Per-column top-2 of a power row (MODE 3 of m4_rows2): the column k1 holds the
// samples k1 + N1 k2, N1 apart, so when 2 spc - 1 <= N1 the open window around the
// row's argmax holds at most one of them and {a1, first index, runner-up} per column
// give the second peak exactly (g_stats1_kernel's argument with columns for threads).
struct M4Top {
  double a1, a2;
  int ak, pad;
};
// merge the top-2 of a disjoint set into (a1, ak, a2): ties keep the first index
__device__ __forceinline__ void top2_merge(double& a1, int& ak, double& a2, double b1, int bk,
                                           double b2) {
  const bool take = better(b1, bk, a1, ak);
  a2 = take ? fmax(a1, b2) : fmax(a2, b1);
  ak = take ? bk : ak;
  a1 = take ? b1 : a1;
}

// push one sample into (a1, ak, a2): top2_merge with b2 = -1, in 5 VALU operations
// (a2 = max(a2, min(v, a1)) holds whether or not v takes the lead)
__device__ __forceinline__ void top1_push(double& a1, int& ak, double& a2, double v, int k) {
  const bool take = v > a1 || (v == a1 && k < ak);
  a2 = fmax(a2, fmin(v, a1));
  ak = take ? k : ak;
  a1 = fmax(a1, v);
}

// one wave: the statistics of unit u0 + r from its per-column top-2 rows
__device__ __forceinline__ void m4_stats_row(const M4Top* __restrict__ top, int r, int N1, int N,
                                             int u0, int n_blocks, int nc, int spc,
                                             gnsscorr_acq_row* __restrict__ stats) {
  const int lane = threadIdx.x % 64;
  const int unit = u0 + r;
  const M4Top* t = top + (long)r * N1;
  const int rowid = nc ? unit : unit / n_blocks;
  const int blk0 = nc ? 0 : unit % n_blocks;
  double bv = -1.0;
  int bk = INT_MAX;
  for (int c = lane; c < N1; c += 64)
    if (better(t[c].a1, t[c].ak, bv, bk)) { bv = t[c].a1; bk = t[c].ak; }
  wave_argmax(bv, bk);
  double sv = -1.0;
  for (int c = lane; c < N1; c += 64) {
    int d = t[c].ak - bk;
    d += d < 0 ? N : 0;
    sv = fmax(sv, (d >= spc && d <= N - spc) ? t[c].a1 : t[c].a2);
  }
  sv = wave_max(sv);
  if (lane == 0) {
    gnsscorr_acq_row o;
    o.peak = bv;
    o.second = sv;
    o.argmax = bk;
    o.block = nc ? -1 : blk0;
    stats[(long)rowid * n_blocks + blk0] = o;
  }
}

__global__ __launch_bounds__(64) void m4_stats_kernel(const M4Top* __restrict__ top, int N1,
                                                      int N, int u0, int n_blocks, int nc,
                                                      int spc,
                                                      gnsscorr_acq_row* __restrict__ stats) {
  m4_stats_row(top, blockIdx.x, N1, N, u0, n_blocks, nc, spc, stats);
}

// A chunk's statistics pass carried by the next chunk's first m4_cols2 launch: extra
// rows of workgroups (one statistics row per wave) after the main grid.  Stream order
// puts them after the chunk's last m4_rows2 (which wrote top) and before the next
// chunk's (which overwrites it); it saves one launch and its tail per chunk.
struct M4StatsJob {
  const M4Top* top = nullptr;
  gnsscorr_acq_row* stats = nullptr;
  int n = 0, u0 = 0, N1 = 0, n_blocks = 1, nc = 0, spc = 0;
  int main_rows = 0;   // the launch's own rows (blockIdx.y below: the column pass)
};

// The column pass without its first and last LDS round trips (round 6): the A-point
// stage reads its inputs (or forms the correlation product) straight from global
// memory -- a lane's task is (q, t), 64 lanes cover 4 values of q x 16 consecutive
// columns, whole 256-byte runs -- and the B-point stage writes its outputs, times
// W_N^(n2 k1), straight to Y.  The LDS holds only the exchange between the stages, one
// fp64 plane at a time (real parts, then imaginary parts: 15.2 KB per tile, 126 VGPRs,
// 16 waves per CU; complex, 30.5 KB held it to 10).
template <int A, int B, int MODE>
__global__ __launch_bounds__(kM4ColThreads) M4_COLS2_ATTR void m4_cols2(const v2d* __restrict__ in, int in_rs,
                                                        v2d* __restrict__ out, int N,
                                                        const v2d* __restrict__ tw,
                                                        const v2d* __restrict__ tws, MixCorr cp,
                                                        M4StatsJob sj) {
  constexpr int N1 = A * B;
  static_assert(kM4ColThreads % kM4T2 == 0, "m4_cols2: a lane keeps one column");
  if ((int)blockIdx.y >= sj.main_rows) {   // the previous chunk's statistics (whole workgroups)
    const int r = (((int)blockIdx.y - sj.main_rows) * (int)gridDim.x + (int)blockIdx.x) *
                      (kM4ColThreads / 64) + (int)threadIdx.x / 64;
    if (r < sj.n) m4_stats_row(sj.top, r, sj.N1, N, sj.u0, sj.n_blocks, sj.nc, sj.spc, sj.stats);
    return;
  }
#if M4_COLS2_PLANE
  __shared__ double sp[N1][kM4T2 + 1];   // one fp64 plane: real parts, then imaginary
#else
  __shared__ v2d s[N1][kM4T2 + 1];
#endif
  const int N2 = N / N1;
  const int n2_0 = blockIdx.x * kM4T2;
  const long row = blockIdx.y;
  const int t = threadIdx.x % kM4T2, n2 = n2_0 + t;
  const bool col = n2 < N2;
  const v2d *Xr = nullptr, *Fr = nullptr;
  int shift = 0;
  if constexpr (MODE == 1) mix_unit_rows(cp, cp.u0 + (int)row, Xr, Fr, shift);
  // ---- stage A: task (q, t), q = (task / kM4T2) < B: the A-point DFT over p of
  // x[B p + q], times W_N1^(q u), into LDS slot B u + q
  constexpr int kLanesQ = kM4ColThreads / kM4T2;   // values of q per pass
  constexpr int kItA = (B + kLanesQ - 1) / kLanesQ;
#if M4_COLS2_PLANE
  double ai[kItA][A];
#endif
#pragma unroll
  for (int it = 0; it < kItA; it++) {
    const int q = threadIdx.x / kM4T2 + kLanesQ * it;
    if (q >= B) continue;
    v2d v[A];
#pragma unroll
    for (int p = 0; p < A; p++) {
      const int n = N2 * (B * p + q) + n2;
      if constexpr (MODE == 1) {
        int sx = n - shift;
        sx += sx < 0 ? N : 0;
        const v2d xv = col ? Xr[sx] : (v2d){0.0, 0.0}, f = col ? Fr[n] : (v2d){0.0, 0.0};
        v[p] = (v2d){fma(xv.x, f.x, xv.y * f.y), fma(xv.x, f.y, -(xv.y * f.x))};   // conj(X) F
      } else {
        v[p] = col ? in[row * in_rs + n] : (v2d){0.0, 0.0};
      }
    }
    dft<A>(v);
#pragma unroll
    for (int u = 1; u < A; u++) v[u] = cmul(v[u], tws[q * u]);   // W_N1^(q u), q u < N1
#if M4_COLS2_PLANE
#pragma unroll
    for (int u = 0; u < A; u++) {
      sp[B * u + q][t] = v[u].x;
      ai[it][u] = v[u].y;
    }
#else
#pragma unroll
    for (int u = 0; u < A; u++) s[B * u + q][t] = v[u];
#endif
  }
  __syncthreads();
  // ---- stage B: task (u, t), u = threadIdx.x / kM4T2 < A: the B-point DFT over q;
  // output w is k1 = u + A w, times W_N^(n2 k1) = W_N^(n2 u) (W_N^(A n2))^w
  constexpr int kItB = (A + kLanesQ - 1) / kLanesQ;
#if M4_COLS2_PLANE
  static_assert(kItB == 1, "m4_cols2: one B-point pass (the plane exchange)");
  v2d vb[B];
  {
    const int u = threadIdx.x / kM4T2;
#pragma unroll
    for (int q = 0; q < B; q++) vb[q].x = u < A ? sp[B * u + q][t] : 0.0;
  }
  __syncthreads();   // the imaginary parts overwrite the plane
#pragma unroll
  for (int it = 0; it < kItA; it++) {
    const int q = threadIdx.x / kM4T2 + kLanesQ * it;
    if (q < B) {
#pragma unroll
      for (int u = 0; u < A; u++) sp[B * u + q][t] = ai[it][u];
    }
  }
  __syncthreads();
  {
    const int u = threadIdx.x / kM4T2;
#pragma unroll
    for (int q = 0; q < B; q++) vb[q].y = u < A ? sp[B * u + q][t] : 0.0;
  }
#endif
#pragma unroll
  for (int it = 0; it < kItB; it++) {
    const int u = threadIdx.x / kM4T2 + kLanesQ * it;
    if (u >= A) continue;
#if M4_COLS2_PLANE
    v2d (&v)[B] = vb;
#else
    v2d v[B];
#pragma unroll
    for (int q = 0; q < B; q++) v[q] = s[B * u + q][t];
#endif
    dft<B>(v);
    if (col) {
      v2d wc = tw[n2 * u], ws = tw[A * n2];   // n2 u < N, A n2 < N
      const long base = row * (long)N1 * m4_pitch(N2) + n2;
#pragma unroll
      for (int w = 0; w < B; w++) {
        out[base + (long)(u + A * w) * m4_pitch(N2)] = cmul(v[w], wc);
        wc = cmul(wc, ws);
      }
    }
  }
}

// m4_rows2 MODE 0: complex rows out (stride out_rs); MODE 2: |.|^2 / N^2 into pw (added
// to the running sums when ACC); MODE 3: as 2 on a row's last block, per-column top-2
// into top (the power row is not stored)
// The rows pass (round 6; the round-5 m4_rows kept complex rows in LDS, 21.9 KB per
// 4-row tile, 7 waves per CU): the C-point stage reads its inputs straight from Y
// (lanes cover 4 rows x 16 consecutive n2: whole lines), the exchange to the D-point
// stage goes through ONE fp64 plane at a time (real parts, then imaginary parts:
// 4 x (N2 + 1) doubles, 10.9 KB), and the prime D-point stage emits its outputs as
// they are formed (power, statistics or complex rows go out from registers, no LDS
// round trip).  164 VGPRs: 12 waves per CU.  The arithmetic is m4_rows' except the
// stage-A twiddles (a recurrence, <= C roundings of drift).  38.192 Msps search
// 1.14-1.15 -> 1.09-1.11 ms (profiles/r6/acq_generic_rows2_ab_r7b.log).
#ifndef M4_ROWS2_WPE
#define M4_ROWS2_WPE 3   // waves per SIMD of m4_rows2 (164 VGPRs)
#endif
#ifndef M4_ROWS2_ROWS
#define M4_ROWS2_ROWS 4   // rows k1 per m4_rows2 workgroup (2: 150 VGPRs, 12 waves per CU, but
                          // 22 of 64 lanes in the 31-point stage: 1.21 against 1.10 ms)
#endif
constexpr int kR2 = M4_ROWS2_ROWS;
template <int C, int D, int MODE, bool ACC>
__global__ __launch_bounds__(kM4RowThreads) __attribute__((amdgpu_waves_per_eu(M4_ROWS2_WPE)))
void m4_rows2(const v2d* __restrict__ Y, v2d* __restrict__ out, int out_rs, int N,
              const v2d* __restrict__ tws, double* __restrict__ pw, int acc,
              M4Top* __restrict__ top) {
  constexpr int N2 = C * D, P2 = m4_pitch(C * D);
  static_assert(is_prime(D), "m4_rows2: the second stage emits a prime DFT's outputs");
  static_assert(kM4RowThreads == 64 && D * kR2 <= 3 * 64 && C * kR2 <= 64,
                "m4_rows2: up to three stage-A passes, one stage-B pass per wave");
  // plane pitch (doubles): LP = 8 mod 32, so the 32 lanes of a half-wave (4 rows x 8
  // consecutive q, or 4 rows x 8 values of u) fall on 32 distinct bank pairs (at
  // N2 + 1 = 342 the rows overlapped: 44 % of the LDS cycles were bank conflicts)
  constexpr int LP = N2 + 1 + ((8 - (N2 + 1)) % 32 + 32) % 32;
  static_assert(LP % 32 == 8 && LP > N2, "m4_rows2: plane pitch");
  __shared__ double sp[kR2][LP];
  const int N1 = N / N2;
  const int k1_0 = blockIdx.x * kR2;
  const long row = blockIdx.y;
  const int t = threadIdx.x;
  const v2d* Yt = Y + row * (long)N1 * P2 + (long)k1_0 * P2;
  // ---- stage A: task (q, r) = (task / kR2, task % kR2), the C-point DFT over p of
  // Y[k1_0 + r][D p + q], then W_N2^(q u).  One pass after the other, each pass's real
  // parts into the plane as soon as they exist: only the imaginary parts stay live
  // (the other waves of the CU hide the load latency)
  constexpr int kTA = D * kR2, kItA = (kTA + 63) / 64;
  // the passes as a loop that is NOT unrolled: unrolled, the scheduler overlapped
  // them (232 VGPRs, 2 waves per SIMD); as a loop, 164 VGPRs: 3 waves per SIMD
  double ai[kItA][C];
#pragma unroll 1
  for (int it = 0; it < kItA; it++) {
    const int task = t + 64 * it, q = task / kR2, r = task % kR2;
    const bool ok = task < kTA && k1_0 + r < N1;
    v2d v[C];
#pragma unroll
    for (int p = 0; p < C; p++) v[p] = ok ? Yt[(long)r * P2 + D * p + q] : (v2d){0.0, 0.0};
    dft<C>(v);
    // W_N2^(q u) = (W_N2^q)^u by recurrence: one table load per task instead of C - 1
    // (all hoisted, they doubled the pass's live registers); <= C roundings of drift
    const v2d w1 = tws[q < D ? q : 0];
    v2d wu = w1;
#pragma unroll
    for (int u = 1; u < C; u++) {
      v[u] = cmul(v[u], wu);
      wu = cmul(wu, w1);
    }
#pragma unroll
    for (int u = 0; u < C; u++) {
      if (task < kTA) sp[r][D * u + q] = v[u].x;
      if (it == 0) ai[0][u] = v[u].y;   // (constant register indices: uniform branches)
      else if (kItA < 3 || it == 1) ai[kItA > 1 ? 1 : 0][u] = v[u].y;
      else ai[kItA - 1][u] = v[u].y;
    }
    // the next pass's loads and arithmetic stay behind this one (interleaving the two
    // passes, the scheduler held both passes' working sets)
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  // ---- exchange, one plane at a time; stage B: task (u, r) = (t / kR2, t % kR2)
  const int ub = t / kR2, rb = t % kR2;
  const bool actB = ub < C && k1_0 + rb < N1;
  // the exchange reads are not predicated: an inactive lane reads a valid slot (ub
  // clamped) and runs the D-point DFT on it, but emits nothing
  const int ubc = min(ub, C - 1);
  v2d x[D];
  __syncthreads();
#pragma unroll
  for (int w = 0; w < D; w++) x[w].x = sp[rb][D * ubc + w];
  __syncthreads();   // the imaginary parts overwrite the plane
#pragma unroll
  for (int it = 0; it < kItA; it++) {
    const int task = t + 64 * it, q = task / kR2, r = task % kR2;
    if (task < kTA) {
#pragma unroll
      for (int u = 0; u < C; u++) sp[r][D * u + q] = ai[it][u];
    }
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < D; w++) x[w].y = sp[rb][D * ubc + w];
  __builtin_amdgcn_sched_barrier(0);
  // ---- stage B: the D-point DFT; output w is element k2 = ub + C w of column k1
  const int k1 = k1_0 + rb;
  const double sc = 1.0 / ((double)N * (double)N);
  double a1 = -1.0, a2 = -1.0;
  int ak = INT_MAX;
  auto emit = [&](int w, v2d v) {
    if (!actB) return;
    const int d = k1 + N1 * (ub + C * w);   // < N
    if constexpr (MODE == 2 || MODE == 3) {
      const double q = fma(v.x, v.x, v.y * v.y) * sc;
      double* o = pw + row * N + d;
      const double val = ACC ? *o + q : q;   // (ACC: the running sums of earlier blocks)
      if constexpr (MODE == 2) *o = val;
      else top1_push(a1, ak, a2, val, d);    // (the row's power is not stored)
    } else {
      out[row * out_rs + d] = v;
    }
  };
  dft_prime_emit<D, true>(x, emit);
  if constexpr (MODE == 3) {
    // the column's C tasks sit in the lanes rb + kR2 u: a tree over u (step s merges
    // the disjoint lane ranges [u, u + s) and [u + s, u + 2 s) within the column)
#pragma unroll
    for (int st = 1; st < C; st <<= 1) {
      const double b1 = __shfl_down(a1, kR2 * st, 64), b2 = __shfl_down(a2, kR2 * st, 64);
      const int bk = __shfl_down(ak, kR2 * st, 64);
      if (ub + st < C) top2_merge(a1, ak, a2, b1, bk, b2);
    }
    if (t < kR2 && k1_0 + t < N1) top[row * N1 + k1_0 + t] = M4Top{a1, a2, ak, 0};
  }
}

// Row statistics from the per-column top-2 (one wave per row): the argmax over the
// columns, then the second peak as the maximum of each column's a1 when its argmax lies
// outside the open circular window (argmax - spc, argmax + spc), else its runner-up.
// Same results as g_stats1_kernel on the power rows.

// the compiled four-step plans: {A, B, C, D}
constexpr int kM4Plans[][4] = {{0, 0, 0, 0}, {7, 16, 11, 31}, {3, 16, 11, 31}};

int m4_plan(int N) {
  for (int i = 1; i < (int)(sizeof kM4Plans / sizeof kM4Plans[0]); i++)
    if (N == kM4Plans[i][0] * kM4Plans[i][1] * kM4Plans[i][2] * kM4Plans[i][3]) return i;
  return 0;
}

// rows [src] -> DFT rows or the correlation's power rows, one chunk of `rows`
template <int MODE_IN, int MODE_OUT>
int m4_launch(gnsscorr_acq_ctx* c, const v2d* in, int in_rs, v2d* out, int out_rs, int rows,
              const MixCorr& cp, double* pw, int acc,
              const M4StatsJob* stats_job = nullptr, int lane = 0,
              hipEvent_t after_cols = nullptr) {
  const int N = c->cfg.n_samples;
  M4StatsJob sj = stats_job ? *stats_job : M4StatsJob{};
  sj.main_rows = rows;
  const int per_y = (N / (kM4Plans[c->m4][0] * kM4Plans[c->m4][1]) + kM4T2 - 1) / kM4T2 *
                    (kM4ColThreads / 64);   // statistics rows per extra grid row
  const int ey = sj.n > 0 ? (sj.n + per_y - 1) / per_y : 0;
  const v2d* tw = (const v2d*)c->d_twN;
  const v2d* tws1 = (const v2d*)c->d_twm4;   // W_N1^j, then W_N2^j from + N1
  v2d* Y = (v2d*)(lane ? c->d_gA2 : c->d_gA);
  M4Top* top = (M4Top*)(lane ? c->d_m4top2 : c->d_m4top);
  hipStream_t st = lane ? c->m4_s2 : c->stream;
  switch (c->m4) {
#define M4_CASE(I, A, B, C, D)                                                                 \
  case I:                                                                                      \
    hipLaunchKernelGGL((m4_cols2<A, B, MODE_IN>),                                              \
                       dim3((N / (A * B) + kM4T2 - 1) / kM4T2, rows + ey), dim3(kM4ColThreads), \
                       0, st, in, in_rs, Y, N, tw, tws1, cp, sj);                              \
    if (after_cols) HIP_TRY(hipEventRecord(after_cols, st));                                   \
    if (acc)                                                                                   \
      hipLaunchKernelGGL((m4_rows2<C, D, MODE_OUT, true>), dim3((A * B + kR2 - 1) / kR2, rows),   \
                         dim3(kM4RowThreads), 0, st, Y, out, out_rs, N, tws1 + A * B, pw,        \
                         acc, top);                                                            \
    else                                                                                       \
      hipLaunchKernelGGL((m4_rows2<C, D, MODE_OUT, false>), dim3((A * B + kR2 - 1) / kR2, rows),  \
                         dim3(kM4RowThreads), 0, st, Y, out, out_rs, N, tws1 + A * B, pw,        \
                         acc, top);                                                            \
    break;
    M4_CASE(1, 7, 16, 11, 31)
    M4_CASE(2, 3, 16, 11, 31)
#undef M4_CASE
    default:
      gnsscorr_set_error("acq64 four-step: no plan %d", c->m4);
      return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

// DFT_N of `rows` natural rows a (stride src_rs) -> out (stride rs), chunked
int mx_dft_rows(gnsscorr_acq_ctx* c, const v2d* a, int src_rs, int rows, v2d* out, int rs) {
  const int N = c->cfg.n_samples, P = c->mix_nr;
  const MixCorr none{};
  for (int r0 = 0; r0 < rows; r0 += c->g_chunk) {
    const int nr = rows - r0 < c->g_chunk ? rows - r0 : c->g_chunk;
    if (c->m4) {
      const int rc = m4_launch<0, 0>(c, a + (long)r0 * src_rs, src_rs, out + (long)r0 * rs, rs, nr,
                                     none, nullptr, 0);
      if (rc) return rc;
      continue;
    }
    v2d *A = (v2d*)c->d_gA, *B = (v2d*)c->d_gB;
    const v2d* src = a + (long)r0 * src_rs;
    int srs = src_rs, Ns = 1;
    for (int i = 0; i < P; i++) {
      const bool last = i + 1 == P;
      v2d* dst = last ? out + (long)r0 * rs : (i % 2 == 0 ? A : B);
      int rc = mx_launch<0>(c, c->mix_r[i], src, srs, dst, last ? rs : N, nr, Ns, none, nullptr, 0);
      if (rc) return rc;
      src = dst;
      srs = N;
      Ns *= c->mix_r[i];
    }
  }
  return GNSSCORR_OK;
}

int mx_correlate(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_groups, int n_bins,
                 const int32_t* d_gcode, const int32_t* d_gfreq, int spc, double* d_dump,
                 int dump_block) {
  const int N = c->cfg.n_samples, P = c->mix_nr;
  const bool nc = mode == GNSSCORR_ACQ_NONCOHERENT;
  // records: every group on every record of the resident spectra (virtual groups)
  const int nrec = c->spec_recs;
  const int n_units = nrec * n_groups * n_bins * (nc ? 1 : n_blocks);
  // four-step plans: the row statistics ride on the last block's m4_rows2 (per-column
  // top-2; its power rows are then not stored) unless the window can hold two samples
  // of a column or the power rows are dumped
  const int N1 = c->m4 ? kM4Plans[c->m4][0] * kM4Plans[c->m4][1] : 0;
  const bool fused = c->m4 && c->d_m4top && 2 * spc - 1 <= N1 && !d_dump;
  // equal chunks (7 x 375 rows rather than 6 x 385 + 314 at the bench's 2 624); with
  // two lanes an even count, chunk i on lane i % 2 (stream, Y, power rows, top-2 of
  // its own), forked from and joined back to the context stream
  const int lanes = c->m4 ? c->m4_lanes : 1;
  int n_ch = (n_units + c->g_chunk - 1) / c->g_chunk;
  if (lanes == 2 && n_ch > 1 && n_ch % 2) n_ch++;
  const int step = n_ch > 0 ? (n_units + n_ch - 1) / n_ch : c->g_chunk;
  // lane 1 starts after lane 0's first column pass, so from then on one lane's column
  // pass (memory-bound) runs beside the other's row pass (fp64-issue-bound); started
  // together, the lanes ran the same pass at the same time
  M4StatsJob pends[2];   // per lane: fused statistics of its previous chunk, not yet launched
  int ci = 0;
  for (int u0 = 0; u0 < n_units; u0 += step, ci++) {
    const int nu = n_units - u0 < step ? n_units - u0 : step;
    const int nb = nc ? n_blocks : 1;
    const int lane = lanes == 2 ? ci % 2 : 0;
    M4StatsJob& pend = pends[lane];
    double* const pw = lane ? c->d_gpw2 : c->d_gpw;
    hipStream_t const st = lane ? c->m4_s2 : c->stream;
    if (lanes == 2 && ci == 1) HIP_TRY(hipStreamWaitEvent(c->m4_s2, c->m4_ev[0], 0));
    for (int b = 0; b < nb; b++) {
      MixCorr cp{(const v2d*)c->d_X64, (const v2d*)c->d_F64, c->rs64, n_blocks, nc ? b : -1,
                 n_bins, u0, d_gcode, d_gfreq, (const int2*)c->d_fmap64, n_groups,
                 n_blocks * nrec};
      if (c->m4) {
        const M4StatsJob* sj = b == 0 && pend.n > 0 ? &pend : nullptr;
        hipEvent_t const fork = lanes == 2 && ci == 0 && b == 0 ? c->m4_ev[0] : nullptr;
        const int rc =
            fused && b == nb - 1
                ? m4_launch<1, 3>(c, nullptr, 0, nullptr, 0, nu, cp, pw, b > 0, sj, lane, fork)
                : m4_launch<1, 2>(c, nullptr, 0, nullptr, 0, nu, cp, pw, b > 0, sj, lane, fork);
        if (rc) return rc;
        if (sj) pend.n = 0;
        continue;
      }
      v2d *A = (v2d*)c->d_gA, *B = (v2d*)c->d_gB;
      const v2d* src = nullptr;
      int Ns = 1;
      for (int i = 0; i < P; i++) {
        v2d* dst = i % 2 == 0 ? A : B;
        int rc = i == 0 ? mx_launch<1>(c, c->mix_r[i], nullptr, 0, dst, N, nu, Ns, cp, nullptr, 0)
                 : i + 1 == P ? mx_launch<2>(c, c->mix_r[i], src, N, nullptr, 0, nu, Ns, cp,
                                             c->d_gpw, b > 0)
                              : mx_launch<0>(c, c->mix_r[i], src, N, dst, N, nu, Ns, cp, nullptr, 0);
        if (rc) return rc;
        src = dst;
        Ns *= c->mix_r[i];
      }
    }
    if (fused) {   // carried by the lane's next column pass, or launched below
      pend.top = (const M4Top*)(lane ? c->d_m4top2 : c->d_m4top);
      pend.stats = c->d_stats;
      pend.n = nu;
      pend.u0 = u0;
      pend.N1 = N1;
      pend.n_blocks = n_blocks;
      pend.nc = (int)nc;
      pend.spc = spc;
    } else if (stats1_exact(N, spc))
      hipLaunchKernelGGL(g_stats1_kernel, dim3(nu), dim3(kStatsThreads), 0, st,
                         (const double*)pw, N, u0, n_blocks, (int)nc, spc, c->d_stats,
                         d_dump, dump_block);
    else
      hipLaunchKernelGGL(g_stats_kernel, dim3(nu), dim3(kGThreads), 0, st,
                         (const double*)pw, N, u0, n_blocks, (int)nc, spc, c->d_stats,
                         d_dump, dump_block);
    HIP_TRY(hipGetLastError());
  }
  for (int l = 0; l < 2; l++)
    if (pends[l].n > 0) {   // each lane's last chunk's statistics
      hipLaunchKernelGGL(m4_stats_kernel, dim3(pends[l].n), dim3(64), 0,
                         l ? c->m4_s2 : c->stream, pends[l].top, N1, N, pends[l].u0, n_blocks,
                         (int)nc, spc, c->d_stats);
      HIP_TRY(hipGetLastError());
    }
  if (lanes == 2) {
    HIP_TRY(hipEventRecord(c->m4_ev[1], c->m4_s2));
    HIP_TRY(hipStreamWaitEvent(c->stream, c->m4_ev[1], 0));
  }
  return GNSSCORR_OK;
}

int mx_init(gnsscorr_acq_ctx* c) {
  const long N = c->cfg.n_samples;
  // (the four-step plan's Y rows at the m4_pitch, a few % above N)
  const long ya = c->m4 ? (long)kM4Plans[c->m4][0] * kM4Plans[c->m4][1] *
                              m4_pitch((int)(N / (kM4Plans[c->m4][0] * kM4Plans[c->m4][1])))
                        : N;
  // Rows per chunk from the work buffer's size.  Large chunks keep each pass at ~10 k
  // workgroups (64 MiB: 25 chunks per search, 1.72 against 1.38 ms, round 5,
  // profiles/r5/acq_generic_chunk_ab_r5ao.log).  The four-step plan's Y is written by
  // m4_cols2 and read back at once by m4_rows2: at <= 232 MiB (385 rows at N = 38 192)
  // it stays in the 256 MB memory-side cache between the two passes.  A sweep of the
  // chunk size gave 0.963-0.965 ms at 242 MB of Y, 1.005 ms at 277 MB (the round-5 size)
  // and 1.007-1.028 ms at 259 MB (profiles/r6/acq_generic_chunk_sweep_r7h.log).
  // GNSSCORR_ACQ_GCHUNK_MB: another size in MiB, for A/Bs.
  // Two chunk lanes (four-step plan; GNSSCORR_ACQ_M4LANES=1: one) split that budget:
  // 116 MiB of Y each, so both lanes' Y stay in the cache together, and one chunk's
  // column pass (memory-bound) overlaps the other's row pass (fp64-issue-bound).  Two
  // whole searches on two streams ran 0.783-0.785 ms per search against 0.903-0.908 ms
  // on one (profiles/r6/acq_generic_overlap_r8c.log); the lanes of one search gain
  // 3 % (0.906-0.912 against 0.930-0.946 ms; 58 / 87 / 145 / 232 MiB per lane chunk
  // slower, profiles/r6/acq_generic_lanes_ab_r8f.log): the search's own set-up and
  // selection still run alone before the fork and after the join.
  const char* gl = getenv("GNSSCORR_ACQ_M4LANES");
  c->m4_lanes = c->m4 && !(gl && gl[0] == '1') ? 2 : 1;
  const char* gm = getenv("GNSSCORR_ACQ_GCHUNK_MB");
  const long mb = gm && atol(gm) > 0 ? atol(gm) : (c->m4 ? 232 / c->m4_lanes : 256);
  c->g_chunk = chunk_cap(c, (int)((mb << 20) / (ya * 16)));
  HIP_TRY(hipMalloc(&c->d_twN, sizeof(double2) * N));
  HIP_TRY(hipMalloc(&c->d_gA, sizeof(double2) * (size_t)ya * c->g_chunk));
  if (!c->m4)   // the four-step plan's passes need one work buffer (Y), the Stockham passes two
    HIP_TRY(hipMalloc(&c->d_gB, sizeof(double2) * (size_t)N * c->g_chunk));
  HIP_TRY(hipMalloc(&c->d_gpw, sizeof(double) * (size_t)N * c->g_chunk));
  // GNSSCORR_ACQ_M4STATS=0: the four-step plan keeps the separate statistics pass
  const char* fs = getenv("GNSSCORR_ACQ_M4STATS");
  const size_t top_bytes = sizeof(M4Top) * (size_t)(c->m4 ? kM4Plans[c->m4][0] * kM4Plans[c->m4][1] : 0) *
                           c->g_chunk;
  if (c->m4 && !(fs && fs[0] == '0')) HIP_TRY(hipMalloc(&c->d_m4top, top_bytes));
  if (c->m4_lanes == 2) {
    HIP_TRY(hipMalloc(&c->d_gA2, sizeof(double2) * (size_t)ya * c->g_chunk));
    HIP_TRY(hipMalloc(&c->d_gpw2, sizeof(double) * (size_t)N * c->g_chunk));
    if (c->d_m4top) HIP_TRY(hipMalloc(&c->d_m4top2, top_bytes));
    HIP_TRY(hipStreamCreateWithFlags(&c->m4_s2, hipStreamNonBlocking));
    for (hipEvent_t& ev : c->m4_ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  }
  double2* h = (double2*)malloc(sizeof(double2) * N);
  if (!h) return GNSSCORR_ENOMEM;
  for (long t = 0; t < N; t++) {   // W_N^t = exp(-2 pi i t / N)
    const double a = -2.0 * M_PI * ((double)t / (double)N);
    h[t] = make_double2(cos(a), sin(a));
  }
  hipError_t e = hipMemcpy(c->d_twN, h, sizeof(double2) * N, hipMemcpyHostToDevice);
  if (e == hipSuccess && c->m4) {
    // the passes' inner twiddles as compact tables (the same values as d_twN's)
    const long N1 = kM4Plans[c->m4][0] * kM4Plans[c->m4][1], N2 = N / N1;
    double2* ht = (double2*)malloc(sizeof(double2) * (N1 + N2));
    if (!ht) { free(h); return GNSSCORR_ENOMEM; }
    for (long j = 0; j < N1; j++) ht[j] = h[j * N2];        // W_N1^j = W_N^(j N2)
    for (long j = 0; j < N2; j++) ht[N1 + j] = h[j * N1];   // W_N2^j = W_N^(j N1)
    e = hipMalloc(&c->d_twm4, sizeof(double2) * (N1 + N2));
    if (e == hipSuccess)
      e = hipMemcpy(c->d_twm4, ht, sizeof(double2) * (N1 + N2), hipMemcpyHostToDevice);
    free(ht);
  }
  free(h);
  HIP_TRY(e);
  return GNSSCORR_OK;
}

}  // namespace

int acq64_plan_for(int n_samples) {
  // GNSSCORR_ACQ_GENERIC=1: the Bluestein engine for every N (cross-checks)
  const char* fg = getenv("GNSSCORR_ACQ_GENERIC");
  const int force_generic = fg ? atoi(fg) : 0;
  if (!force_generic && n_samples == PlanA::N) return 1;
  if (!force_generic && n_samples == PlanB::N) return 2;
  if (n_samples >= 64 && n_samples <= (1 << 19)) return 3;
  return 0;
}

namespace {
int mix_factor(int N, int* r);
int m4_plan(int N);
int mx_init(gnsscorr_acq_ctx* c);
}  // namespace

int acq64_init(gnsscorr_acq_ctx* c) {
  c->plan64 = acq64_plan_for(c->cfg.n_samples);
  if (!c->plan64) {
    gnsscorr_set_error("acq64: n_samples %d outside [64, %d] (compiled plans: %d, %d; "
                       "Bluestein otherwise)", c->cfg.n_samples, 1 << 19, PlanA::N, PlanB::N);
    return GNSSCORR_EINVAL;
  }
  const int N = c->cfg.n_samples;
  c->rs64 = (N + 63) & ~63;
  HIP_TRY(hipMalloc(&c->d_F64, sizeof(double2) * (size_t)c->rs64 * c->cfg.max_codes));
  HIP_TRY(hipMemset(c->d_F64, 0, sizeof(double2) * (size_t)c->rs64 * c->cfg.max_codes));
  HIP_TRY(hipMalloc(&c->d_fmap64, sizeof(int2) * c->cfg.max_freqs));
  HIP_TRY(hipMalloc(&c->d_lead64, sizeof(int) * c->cfg.max_freqs));
  if (c->plan64 == 3) {
    // the mixed-radix plan unless N has a prime factor above 31 (or
    // GNSSCORR_ACQ_BLUESTEIN=1: the chirp-z engine, for cross-checks)
    const char* fb = getenv("GNSSCORR_ACQ_BLUESTEIN");
    c->mix_nr = (fb && atoi(fb)) ? 0 : mix_factor(N, c->mix_r);
    // the four-step plan where one is compiled for N (GNSSCORR_ACQ_MIX4=0: the
    // mixed-radix passes, for cross-checks)
    const char* f4 = getenv("GNSSCORR_ACQ_MIX4");
    c->m4 = c->mix_nr && !(f4 && f4[0] == '0') ? m4_plan(N) : 0;
    return c->mix_nr ? mx_init(c) : g_init(c);
  }
  HIP_TRY(hipMalloc(&c->d_twN, sizeof(double2) * N));
  double2* tw = (double2*)malloc(sizeof(double2) * N);
  for (int j = 0; j < N; j++) {
    // W_N^j = exp(-2 pi i j / N), argument reduced to [0, pi/4]-accurate libm calls
    const double a = 2.0 * M_PI * ((double)j / (double)N);
    tw[j] = make_double2(cos(a), -sin(a));
  }
  hipError_t e = hipMemcpy(c->d_twN, tw, sizeof(double2) * N, hipMemcpyHostToDevice);
  free(tw);
  HIP_TRY(e);
  return GNSSCORR_OK;
}

void acq64_free(gnsscorr_acq_ctx* c) {
  void* bufs[] = {c->d_F64, c->d_X64,   c->d_in64, c->d_twN, c->d_fmap64, c->d_lead64,
                  c->d_chirp, c->d_vf, c->d_twM, c->d_gA,  c->d_gB,     c->d_gpw,
                  c->d_m4top, c->d_twm4, c->d_gA2, c->d_gpw2, c->d_m4top2};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  c->d_gA2 = nullptr;
  c->d_gpw2 = nullptr;
  c->d_m4top2 = nullptr;
  for (hipEvent_t& ev : c->m4_ev)
    if (ev) {
      (void)hipEventDestroy(ev);
      ev = nullptr;
    }
  if (c->m4_s2) (void)hipStreamDestroy(c->m4_s2);
  c->m4_s2 = nullptr;
  c->d_chirp = c->d_vf = c->d_twM = c->d_gA = c->d_gB = nullptr;
  c->d_gpw = nullptr;
  c->d_m4top = nullptr;
  c->d_twm4 = nullptr;
  c->d_F64 = c->d_X64 = c->d_in64 = c->d_twN = nullptr;
  c->d_fmap64 = nullptr;
  c->d_lead64 = nullptr;
}

namespace {

template <class P>
int set_codes_launch(gnsscorr_acq_ctx* c, const int8_t* d_codes, int n_codes) {
  const long n = (long)n_codes * P::N;
  hipLaunchKernelGGL(acq64_codes_kernel<P>, dim3((n + 255) / 256), dim3(256), 0, c->stream,
                     d_codes, n, (v2d*)c->d_in64);
  HIP_TRY(hipGetLastError());
  return fwd_launch<P>(c, (const v2d*)c->d_in64, nullptr, 1, n_codes, (v2d*)c->d_F64);
}

template <class P>
int spectra_launch(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq, int n_blocks, int n_freqs,
                   const double* d_freqs) {
  constexpr int N = P::N;
  const int rows = n_freqs * n_blocks;   // upper bound: classes <= frequencies
  const double delta = c->cfg.samp_rate / N;
  const int fuse = n_freqs <= kFuseClass ? n_freqs : 0;
  if (!fuse) {
    hipLaunchKernelGGL(acq64_classify_kernel, dim3(1), dim3(1024), 0, c->stream, d_freqs,
                       n_freqs, delta, N, c->d_fmap64, c->d_cfreq, c->d_nclass, c->d_resid,
                       c->d_lead64);
    HIP_TRY(hipGetLastError());
  }
  const long work = (long)rows * N;
  const int grid = (int)((work + 255) / 256 < 2048 ? (work + 255) / 256 : 2048);
  hipLaunchKernelGGL(acq64_wipe_kernel<P>, dim3(grid), dim3(256), 0, c->stream, d_if, iq,
                     n_blocks, c->coh, c->d_cfreq, c->d_nclass, 1.0 / c->cfg.samp_rate,
                     (v2d*)c->d_in64, fuse, d_freqs, delta, c->d_fmap64, c->d_cfreq,
                     c->d_nclass);
  HIP_TRY(hipGetLastError());
  return fwd_launch<P>(c, (const v2d*)c->d_in64, c->d_nclass, n_blocks, rows, (v2d*)c->d_X64);
}

}  // namespace

// Once per context (gnsscorr_acq_create): the input buffer of max_codes code
// transforms, and this file's code object loaded on the device (HIP loads a
// translation unit's kernels on their first use: ~3 ms on the first
// set_prn_codes of a process otherwise; hipFuncGetAttributes loads it).
int acq64_preload(gnsscorr_acq_ctx* c) {
  int rc = acq_grow((void**)&c->d_in64, &c->cap_in64, (size_t)c->cfg.max_codes * c->cfg.n_samples,
                    sizeof(double2));
  if (rc) return rc;
  hipFuncAttributes a;
  HIP_TRY(hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&acq64_classify_kernel)));
  return GNSSCORR_OK;
}

int acq64_set_codes(gnsscorr_acq_ctx* c, const int8_t* d_codes, int n_codes) {
  int rc = acq_grow((void**)&c->d_in64, &c->cap_in64, (size_t)n_codes * c->cfg.n_samples,
                    sizeof(double2));
  if (rc) return rc;
  if (c->plan64 == 3) return g_set_codes(c, d_codes, n_codes);
  return c->plan64 == 1 ? set_codes_launch<PlanA>(c, d_codes, n_codes)
                        : set_codes_launch<PlanB>(c, d_codes, n_codes);
}

int acq64_spectra(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq, int n_blocks, int n_freqs,
                  const double* d_freqs) {
  const size_t rows = (size_t)n_freqs * n_blocks;
  int rc = acq_grow((void**)&c->d_in64, &c->cap_in64, rows * c->cfg.n_samples, sizeof(double2));
  if (rc) return rc;
  rc = acq_grow((void**)&c->d_X64, &c->cap_X64, rows * c->rs64, sizeof(double2));
  if (rc) return rc;
  if (c->plan64 == 3) return g_spectra(c, d_if, iq, n_blocks, n_freqs, d_freqs);
  return c->plan64 == 1 ? spectra_launch<PlanA>(c, d_if, iq, n_blocks, n_freqs, d_freqs)
                        : spectra_launch<PlanB>(c, d_if, iq, n_blocks, n_freqs, d_freqs);
}

int acq64_correlate(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_groups, int n_bins,
                    const int32_t* d_gcode, const int32_t* d_gfreq, int spc, double* d_dump,
                    int dump_block) {
  // n_groups per record; the units of every record of the resident spectra run
  // in one launch (virtual groups rec * n_groups + g)
  const int upr = mode == GNSSCORR_ACQ_NONCOHERENT ? 1 : n_blocks;
  const int n_units = (c->d_group_rec ? 1 : c->spec_recs) * n_groups * n_bins * upr;
  if (c->plan64 == 3)
    return g_correlate(c, n_blocks, mode, n_groups, n_bins, d_gcode, d_gfreq, spc, d_dump,
                       dump_block);
  return c->plan64 == 1 ? corr_launch<PlanA>(c, n_blocks, mode, n_units, n_bins, d_gcode, d_gfreq,
                                             spc, d_dump, dump_block, n_groups)
                        : corr_launch<PlanB>(c, n_blocks, mode, n_units, n_bins, d_gcode, d_gfreq,
                                             spc, d_dump, dump_block, n_groups);
}
