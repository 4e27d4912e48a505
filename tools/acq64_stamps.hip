// tools/acq64_stamps.hip -- diagnostic build of the fp64 acquisition
// correlation kernel with s_memtime stamps at its barriers (thread 0 of each
// workgroup).  Not part of the library.  On the GPU box (tools/acq64_stamps.sh):
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc \
//         -c tools/acq64_stamps.hip -o /tmp/s64.o
//   hipcc --offload-arch=gfx950 /tmp/s64.o <library objects except acq64.o> -o /tmp/s64
// Prints the mean cycles per phase over all workgroups of a config-2 launch.
// Read the SHARES; the stamps perturb the kernel slightly.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
__device__ unsigned long long* g_stamps;
#define ACQ64_STAMP(i)                                                            \
  do {                                                                            \
    if (threadIdx.x == 0) {                                                       \
      unsigned long long _t;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");   \
      g_stamps[blockIdx.x * 16 + (i)] = _t;                                       \
    }                                                                             \
  } while (0)
#include "../gnss-sdr.ru_amd/csrc/acq64.hip"

int main() {
  const int G = 32, B = 41, NB = 2, NCLS = 2, RS = 16384;
  const int units = G * B * NB;
  std::vector<double2> hX((size_t)NCLS * NB * RS), hF((size_t)G * RS);
  srand(1);
  for (auto& v : hX) v = make_double2(rand() / (double)RAND_MAX - 0.5, rand() / (double)RAND_MAX - 0.5);
  for (auto& v : hF) v = make_double2(rand() / (double)RAND_MAX - 0.5, rand() / (double)RAND_MAX - 0.5);
  double2 *dX, *dF;
  int *dgc, *dgf, *dord;
  int2* dfm;
  gnsscorr_acq_row* dst;
  unsigned long long* dstamp;
  (void)hipMalloc(&dX, hX.size() * 16);
  (void)hipMalloc(&dF, hF.size() * 16);
  (void)hipMemcpy(dX, hX.data(), hX.size() * 16, hipMemcpyHostToDevice);
  (void)hipMemcpy(dF, hF.data(), hF.size() * 16, hipMemcpyHostToDevice);
  std::vector<int> gc(G), gf(G * B), ord(units);
  std::vector<int2> fm(B);
  for (int g = 0; g < G; g++) gc[g] = g;
  for (int r = 0; r < G * B; r++) gf[r] = r % B;
  for (int b = 0; b < B; b++) fm[b] = make_int2(b & 1, (b / 2 * 1000) % 16368);   // 500 Hz bins
  for (int u = 0; u < units; u++) ord[u] = u;
  (void)hipMalloc(&dgc, G * 4);
  (void)hipMalloc(&dgf, G * B * 4);
  (void)hipMalloc(&dord, units * 4);
  (void)hipMalloc(&dfm, B * 8);
  (void)hipMalloc(&dst, units * sizeof(gnsscorr_acq_row));
  (void)hipMalloc(&dstamp, (size_t)units * 16 * 8);
  (void)hipMemset(dstamp, 0, (size_t)units * 16 * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dstamp, sizeof(dstamp));
  (void)hipMemcpy(dgc, gc.data(), G * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dgf, gf.data(), G * B * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dord, ord.data(), units * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dfm, fm.data(), B * 8, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int it = 0; it < 3; it++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((acq64_corr_kernel<PlanA, 0, false>), dim3(units), dim3(PlanA::TB), 0, 0,
                       (const v2d*)dX, (const v2d*)dF, RS, NB, dgc, dgf, B, 16, dst,
                       (double*)nullptr, -1, dord, dfm, (const v2d*)nullptr);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
  }
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st((size_t)units * 16);
  (void)hipMemcpy(st.data(), dstamp, st.size() * 8, hipMemcpyDeviceToHost);
  const char* names[] = {"start", "load+mul+dft16, ex1 re write", "ex1 re read", "ex1 im write",
                         "ex1 im read", "dft33, ex2 re write", "ex2 re read", "ex2 im write",
                         "ex2 im read+side", "dft31+leftover+pow+argmax", "second peak"};
  double tot = 0, ph[11] = {0};
  for (int u = 0; u < units; u++) {
    for (int i = 1; i <= 10; i++) ph[i] += (double)(st[u * 16 + i] - st[u * 16 + i - 1]);
    tot += (double)(st[u * 16 + 10] - st[u * 16]);
  }
  printf("kernel %.1f us (stamped), mean cycles per unit %.0f\n", ms * 1e3, tot / units);
  for (int i = 1; i <= 10; i++)
    printf("  %-32s %8.0f  %5.1f %%\n", names[i], ph[i] / units, 100.0 * ph[i] / tot);
  return 0;
}
