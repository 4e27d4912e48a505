// tools/acq_pstamps.hip -- diagnostic build of the pipelined acquisition
// correlation kernel with s_memtime stamps at its phase boundaries, taken by
// lane 0 of every wavefront of every workgroup (role summaries use waves 0
// and 8, the first of each role; the per-wave table shows the slowest).
// Not part of the library; run on the GPU box (tools/pstamps.sh).  Read the
// SHARES, never the run time (stamps serialise the kernel).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
__device__ unsigned long long* g_stamps;
#define ACQ_PSTAMP(it, i)                                                         \
  do {                                                                            \
    if ((threadIdx.x & 63) == 0 && (it) < 16) {                                  \
      unsigned long long _t;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");   \
      g_stamps[((blockIdx.x * 16 + (it)) * 16 + (threadIdx.x >> 6)) * 8 + (i)] = _t; \
    }                                                                             \
  } while (0)
#include "../gnss-sdr.ru_amd/csrc/acq.hip"

int main() {
  const int G = 32, B = 41, R = G * B, NB = 2, U = R * NB, GRID = 256;
  std::vector<float2> hX((size_t)B * NB * NPAD), hF((size_t)G * NPAD);
  srand(1);
  for (auto& v : hX) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  for (auto& v : hF) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  float2 *dX, *dF;
  int *dgc, *dgf, *dord;
  int4* dfm;
  gnsscorr_acq_row* drows;
  unsigned long long* dst;
  (void)hipMalloc(&dX, hX.size() * 8);
  (void)hipMalloc(&dF, hF.size() * 8);
  (void)hipMemcpy(dX, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dF, hF.data(), hF.size() * 8, hipMemcpyHostToDevice);
  std::vector<int> gc(G), gf(R), ord(U);
  std::vector<int4> fm(B);
  for (int g = 0; g < G; g++) gc[g] = g;
  for (int r = 0; r < R; r++) gf[r] = r % B;
  const bool shifted = getenv("SHIFTED") != nullptr;
  for (int b = 0; b < B; b++) fm[b] = shifted ? make_int4(b % 2, 3, 1, 5 * 32 + 7) : make_int4(b, 0, 0, 0);
  build_tile_order(G, B, NB, ord.data());
  (void)hipMalloc(&dgc, G * 4);
  (void)hipMalloc(&dgf, R * 4);
  (void)hipMalloc(&dord, U * 4);
  (void)hipMalloc(&dfm, B * sizeof(int4));
  (void)hipMemcpy(dgc, gc.data(), G * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dgf, gf.data(), R * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dord, ord.data(), U * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dfm, fm.data(), B * sizeof(int4), hipMemcpyHostToDevice);
  (void)hipMalloc(&drows, U * sizeof(gnsscorr_acq_row));
  const size_t NS = (size_t)GRID * 16 * 16 * 8;
  (void)hipMalloc(&dst, NS * 8);
  (void)hipMemset(dst, 0, NS * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dst, sizeof(dst));
  for (int it = 0; it < 3; it++)
    hipLaunchKernelGGL(acq_corr_pipe_kernel, dim3(GRID), dim3(kPipeThreads), 0, 0, dX, dF, NB, dgc,
                       dgf, B, 16, drows, dord, dfm, U);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> st(NS);
  (void)hipMemcpy(st.data(), dst, NS * 8, hipMemcpyDeviceToHost);
  // compute role: 0->1 previous unit's reductions + pass33, 1->2 wait S1,
  //               2->3 radix-31 reads + side copy, 3->4 wait S2, 4->5 radix-31 +
  //               leftover + argmax slots, 5->6 wait S3
  // stream role:  0->1 loads + radix-16, 1->2 wait S1, 2->3 (idle), 3->4 S2,
  //               4->5 row write, 5->6 S3
  const int NI = 6;
  const char* names[6] = {"P1 work", "S1 wait", "P2 work", "S2 wait", "P3 work", "S3 wait"};
  for (int role = 0; role < 2; role++) {
    double tot[6] = {0};
    int n = 0;
    for (int b = 0; b < GRID; b++)
      for (int it = 1; it < 10; it++) {   // steady state, skip the prologue iteration
        const unsigned long long* s = &st[((b * 16 + it) * 16 + role * 8) * 8];
        if (!s[NI]) continue;
        for (int i = 0; i < NI; i++) tot[i] += (double)(s[i + 1] - s[i]);
        n++;
      }
    double all = 0;
    for (int i = 0; i < NI; i++) all += tot[i];
    printf("%s role (%d samples), per unit %.0f cycles\n", role ? "stream" : "compute", n, all / n);
    for (int i = 0; i < NI; i++) printf("  %-10s %8.0f  %5.1f%%\n", names[i], tot[i] / n, 100 * tot[i] / all);
  }
  // unit-to-unit period (stamp 0 of consecutive iterations), compute role
  double per = 0;
  int np = 0;
  for (int b = 0; b < GRID; b++)
    for (int it = 1; it < 9; it++) {
      const unsigned long long a = st[((b * 16 + it) * 16) * 8], c = st[((b * 16 + it + 1) * 16) * 8];
      if (a && c) { per += (double)(c - a); np++; }
    }
  printf("period %.0f cycles per unit\n", per / np);
  // per wave: work of P1 and P3 (stamp 0 -> 1 and 4 -> 5), steady state
  printf("wave  P1work  P3work\n");
  for (int w = 0; w < 16; w++) {
    double p1 = 0, p3 = 0;
    int n = 0;
    for (int b = 0; b < GRID; b++)
      for (int it = 1; it < 10; it++) {
        const unsigned long long* s = &st[((b * 16 + it) * 16 + w) * 8];
        if (!s[6]) continue;
        p1 += (double)(s[1] - s[0]);
        p3 += (double)(s[5] - s[4]);
        n++;
      }
    printf("%4d %7.0f %7.0f\n", w, p1 / n, p3 / n);
  }
  return 0;
}
