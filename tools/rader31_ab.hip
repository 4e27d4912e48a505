// tools/rader31_ab.hip -- A/B of the 31-point complex fp64 DFT that is the last
// stage of acq64_corr_kernel (N = 16368 = 16 x 33 x 31): the symmetric direct
// form the kernel uses (dft_prime<31>, acq64.hip) against a Rader form.
//
// Rader (primitive root g = 3, g^15 = -1 mod 31): with s_j = x_j + x_{31-j},
// d_j = x_j - x_{31-j} (j = 1..15), X_m = A_m - i B_m, X_{31-m} = A_m + i B_m,
//   A_{J(b)} = x_0 + sum_a c[(a+b) mod 15] s_{J(a)}       (cyclic, length 15)
//   B_{J(b)} = sigma_b sum_a sigma_a d_{J(a)} sn~[a+b]     (negacyclic, length 15)
// J(a) = 3^a mod 31 folded to 1..15, sigma = -1 where it was folded,
// c[k] = cos(2 pi 3^k / 31), sn~ the antiperiodic sin(2 pi 3^k / 31).
// Both correlations go through 15-point DFTs (Good-Thomas 3 x 5): the cyclic
// one as (1/15) DFT(DFT(u) . conj(DFT(c))), the negacyclic one the same after
// modulating by zeta^-a (zeta = exp(i pi / 15)) and demodulating by zeta^-b.
//
// The two forms run the same 31-point transform on every thread's 31 complex
// values, REPS times (rescaled by 1/31 each time), for the same data; the run
// reports max relative difference of the outputs, time per DFT, and the VALU
// fp64 instruction counts are read from the ISA (tools/rader31_ab.sh).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

typedef double v2d __attribute__((ext_vector_type(2)));

// compile-time constants, as acq64.hip's kTw (literals in scalar registers)
constexpr double kPi = 3.14159265358979323846264338327950288;
constexpr double poly_sin(double x) {
  double x2 = x * x, term = x, sum = x;
  for (int i = 1; i < 12; i++) { term *= -x2 / (double)((2 * i) * (2 * i + 1)); sum += term; }
  return sum;
}
constexpr double poly_cos(double x) {
  double x2 = x * x, term = 1.0, sum = 1.0;
  for (int i = 1; i < 12; i++) { term *= -x2 / (double)((2 * i - 1) * (2 * i)); sum += term; }
  return sum;
}
struct CS { double c, s; };
constexpr CS cs2pi(long j, long R) {   // cos, sin of 2 pi j / R
  j %= R;
  if (j < 0) j += R;
  const long q = (8 * j) / R, rem = 8 * j - q * R;
  double c = 0, s = 0;
  if ((q & 1) == 0) { const double x = (double)rem / (double)R * (kPi / 4); c = poly_cos(x); s = poly_sin(x); }
  else { const double y = (double)(R - rem) / (double)R * (kPi / 4); c = poly_sin(y); s = poly_cos(y); }
  switch ((q >> 1) & 3) {
    case 0: return CS{c, s};
    case 1: return CS{-s, c};
    case 2: return CS{-c, -s};
    default: return CS{s, -c};
  }
}
constexpr int pow3(int a) { int g = 1; for (int i = 0; i < a; i++) g = g * 3 % 31; return g; }
constexpr int Jf(int a) { return pow3(a) <= 15 ? pow3(a) : 31 - pow3(a); }
constexpr int Sg(int a) { return pow3(a) <= 15 ? 1 : -1; }
struct Tabs {
  double c31[32], s31[32];        // cos / sin (2 pi q / 31)
  double d15r[15], d15i[15];      // (1/15) conj(DFT15(c))
  double e15r[15], e15i[15];      // (1/15) sum_t h_t exp(+2 pi i t k / 15), h_t = sn~[t] zeta^t
  double zr[15], zi[15];          // zeta^-a = exp(-i pi a / 15)
  constexpr Tabs() : c31{}, s31{}, d15r{}, d15i{}, e15r{}, e15i{}, zr{}, zi{} {
    for (int q = 0; q < 32; q++) { c31[q] = cs2pi(q, 31).c; s31[q] = cs2pi(q, 31).s; }
    double c[15] = {}, hr[15] = {}, hi[15] = {};
    for (int a = 0; a < 15; a++) {
      c[a] = cs2pi(pow3(a), 31).c;
      const double sn = cs2pi(pow3(a), 31).s;
      hr[a] = sn * cs2pi(a, 30).c;    // zeta^a
      hi[a] = sn * cs2pi(a, 30).s;
      zr[a] = cs2pi(a, 30).c;
      zi[a] = -cs2pi(a, 30).s;
    }
    for (int k = 0; k < 15; k++) {
      double dr = 0, di = 0, er = 0, ei = 0;
      for (int t = 0; t < 15; t++) {
        const CS w = cs2pi((long)t * k, 15);
        dr += c[t] * w.c; di += c[t] * w.s;
        er += hr[t] * w.c - hi[t] * w.s; ei += hr[t] * w.s + hi[t] * w.c;
      }
      d15r[k] = dr / 15; d15i[k] = di / 15; e15r[k] = er / 15; e15i[k] = ei / 15;
    }
  }
};
constexpr Tabs T{};

__device__ __forceinline__ v2d cmul(v2d a, double br, double bi) {
  return (v2d){fma(a.x, br, -(a.y * bi)), fma(a.x, bi, a.y * br)};
}

// ---- direct symmetric form (acq64.hip dft_prime<31>) ----------------------------
template <int P>
__device__ __forceinline__ void dft_direct(v2d (&x)[P]) {
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
      const double c = T.c31[q], sn = T.s31[q];
      A = (v2d){fma(c, s[j].x, A.x), fma(c, s[j].y, A.y)};
      B = (v2d){fma(sn, d[j].x, B.x), fma(sn, d[j].y, B.y)};
    }
    x[m] = (v2d){A.x + B.y, A.y - B.x};
    x[P - m] = (v2d){A.x - B.y, A.y + B.x};
  }
  x[0] = X0;
}

// ---- 15-point DFT, Good-Thomas 3 x 5 (forward, natural order) ----------------------
__device__ __forceinline__ void dft3(v2d& a, v2d& b, v2d& c) {
  const double h = -0.5, r = 0.86602540378443864676;   // W3 = -1/2 - i sqrt(3)/2
  const v2d t = b + c, u = b - c;
  const v2d m = (v2d){fma(h, t.x, a.x), fma(h, t.y, a.y)};
  a = a + t;
  b = (v2d){fma(r, u.y, m.x), fma(-r, u.x, m.y)};    // m - i r u
  c = (v2d){fma(-r, u.y, m.x), fma(r, u.x, m.y)};    // m + i r u
}
__device__ __forceinline__ void dft5(v2d (&x)[5]) {
  const double c1 = 0.30901699437494742410, c2 = -0.80901699437494742410;
  const double s1 = 0.95105651629515357212, s2 = 0.58778525229247312917;
  const v2d s14 = x[1] + x[4], d14 = x[1] - x[4], s23 = x[2] + x[3], d23 = x[2] - x[3];
  const v2d x0 = x[0];
  const v2d A1 = (v2d){fma(c1, s14.x, fma(c2, s23.x, x0.x)), fma(c1, s14.y, fma(c2, s23.y, x0.y))};
  const v2d A2 = (v2d){fma(c2, s14.x, fma(c1, s23.x, x0.x)), fma(c2, s14.y, fma(c1, s23.y, x0.y))};
  const v2d B1 = (v2d){fma(s1, d14.x, s2 * d23.x), fma(s1, d14.y, s2 * d23.y)};
  const v2d B2 = (v2d){fma(s2, d14.x, -(s1 * d23.x)), fma(s2, d14.y, -(s1 * d23.y))};
  x[0] = x0 + s14 + s23;
  x[1] = (v2d){A1.x + B1.y, A1.y - B1.x};
  x[4] = (v2d){A1.x - B1.y, A1.y + B1.x};
  x[2] = (v2d){A2.x + B2.y, A2.y - B2.x};
  x[3] = (v2d){A2.x - B2.y, A2.y + B2.x};
}
// n = (5 a + 3 b) mod 15 (a < 3, b < 5); k = (10 ka + 6 kb) mod 15
__device__ __forceinline__ void dft15(v2d (&x)[15]) {
  v2d y[3][5];
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 5; b++) y[a][b] = x[(5 * a + 3 * b) % 15];
#pragma unroll
  for (int b = 0; b < 5; b++) dft3(y[0][b], y[1][b], y[2][b]);
#pragma unroll
  for (int a = 0; a < 3; a++) dft5(y[a]);
#pragma unroll
  for (int a = 0; a < 3; a++)
#pragma unroll
    for (int b = 0; b < 5; b++) x[(10 * a + 6 * b) % 15] = y[a][b];
}

__device__ __forceinline__ void dft_rader31(v2d (&x)[31]) {
  v2d u[15], w[15];
  const v2d x0 = x[0];
  v2d X0 = x0;
#pragma unroll
  for (int a = 0; a < 15; a++) {
    const int j = Jf(a);
    const v2d s = x[j] + x[31 - j];
    const v2d d = Sg(a) > 0 ? x[j] - x[31 - j] : x[31 - j] - x[j];
    X0 += s;
    u[a] = s;
    w[a] = a == 0 ? d : cmul(d, T.zr[a], T.zi[a]);
  }
  dft15(u);
  dft15(w);
#pragma unroll
  for (int k = 0; k < 15; k++) {
    u[k] = cmul(u[k], T.d15r[k], T.d15i[k]);
    w[k] = cmul(w[k], T.e15r[k], T.e15i[k]);
  }
  dft15(u);
  dft15(w);
#pragma unroll
  for (int b = 0; b < 15; b++) {
    const v2d A = u[b] + x0;
    v2d B = b == 0 ? w[b] : cmul(w[b], T.zr[b], T.zi[b]);
    if (Sg(b) < 0) B = -B;
    const int m = Jf(b);
    x[m] = (v2d){A.x + B.y, A.y - B.x};
    x[31 - m] = (v2d){A.x - B.y, A.y + B.x};
  }
  x[0] = X0;
}

template <int FORM>
__global__ __launch_bounds__(256) void k31(const v2d* __restrict__ in, v2d* __restrict__ out, int reps) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  v2d x[31];
#pragma unroll
  for (int i = 0; i < 31; i++) x[i] = in[(size_t)t * 31 + i];
  for (int r = 0; r < reps; r++) {
    if (FORM == 0) dft_direct<31>(x);
    else dft_rader31(x);
#pragma unroll
    for (int i = 0; i < 31; i++) x[i] *= (1.0 / 31.0);
  }
#pragma unroll
  for (int i = 0; i < 31; i++) out[(size_t)t * 31 + i] = x[i];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 64;
  const int nthr = 256 * 1024;
  const double pi = 3.14159265358979323846;
  std::vector<double> hin((size_t)nthr * 62);
  srand(7);
  for (auto& v : hin) v = (double)rand() / RAND_MAX - 0.5;
  v2d *din, *da, *db;
  (void)hipMalloc(&din, hin.size() * 8);
  (void)hipMalloc(&da, hin.size() * 8);
  (void)hipMalloc(&db, hin.size() * 8);
  (void)hipMemcpy(din, hin.data(), hin.size() * 8, hipMemcpyHostToDevice);
  // correctness: one transform each
  hipLaunchKernelGGL(k31<0>, dim3(nthr / 256), dim3(256), 0, 0, din, da, 1);
  hipLaunchKernelGGL(k31<1>, dim3(nthr / 256), dim3(256), 0, 0, din, db, 1);
  std::vector<double> ra(hin.size()), rb(hin.size());
  (void)hipMemcpy(ra.data(), da, ra.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(rb.data(), db, rb.size() * 8, hipMemcpyDeviceToHost);
  double md = 0, mx = 0;
  for (size_t i = 0; i < ra.size(); i++) { md = fmax(md, fabs(ra[i] - rb[i])); mx = fmax(mx, fabs(ra[i])); }
  // and the direct form against a plain O(N^2) host DFT for thread 0
  double mh = 0;
  for (int k = 0; k < 31; k++) {
    double sr = 0, si = 0;
    for (int n = 0; n < 31; n++) {
      const double xr = hin[2 * n], xi = hin[2 * n + 1];
      sr += xr * cos(2 * pi * n * k / 31) + xi * sin(2 * pi * n * k / 31);
      si += xi * cos(2 * pi * n * k / 31) - xr * sin(2 * pi * n * k / 31);
    }
    mh = fmax(mh, fmax(fabs(sr / 31 - ra[2 * k]), fabs(si / 31 - ra[2 * k + 1])));
  }
  printf("max |direct - rader| %.3e (max |X| %.3e); direct vs host DFT %.3e\n", md, mx, mh);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int form = 0; form < 2; form++) {
    for (int it = 0; it < 3; it++) {
      (void)hipEventRecord(e0, 0);
      if (form == 0) hipLaunchKernelGGL(k31<0>, dim3(nthr / 256), dim3(256), 0, 0, din, da, reps);
      else hipLaunchKernelGGL(k31<1>, dim3(nthr / 256), dim3(256), 0, 0, din, db, reps);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      printf("%s: %.3f ms for %d x %d DFT31 = %.3f ns per DFT (chip)\n", form ? "rader " : "direct",
             ms, nthr, reps, ms * 1e6 / ((double)nthr * reps));
    }
  }
  return 0;
}
