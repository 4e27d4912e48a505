// tools/acq_stamps.hip -- diagnostic build of the acquisition correlation
// kernel with s_memtime stamps at every phase boundary (thread 0 of each
// workgroup).  Not part of the library; run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ignss-sdr.ru_amd/csrc \
//         tools/acq_stamps.hip gnss-sdr.ru_amd/csrc/common.c -o /tmp/acq_stamps
//   /tmp/acq_stamps
// Prints the mean cycles per phase.  Never quote its run time (the stamps
// serialise the kernel); read the SHARES.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
__device__ unsigned long long* g_stamps;
#define ACQ_STAMP(i)                                                              \
  do {                                                                            \
    if (threadIdx.x == 0) {                                                       \
      unsigned long long _t;                                                      \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");   \
      g_stamps[blockIdx.x * 16 + (i)] = _t;                                       \
    }                                                                             \
  } while (0)
#include "../gnss-sdr.ru_amd/csrc/acq.hip"

int main() {
  const int G = 32, B = 41, R = G * B, NB = 2;
  std::vector<float2> hX((size_t)B * NB * NPAD), hF((size_t)G * NPAD);
  srand(1);
  for (auto& v : hX) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  for (auto& v : hF) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  float2 *dX, *dF;
  int *dgc, *dgf, *dord;
  gnsscorr_acq_row* drows;
  unsigned long long* dst;
  (void)hipMalloc(&dX, hX.size() * 8);
  (void)hipMalloc(&dF, hF.size() * 8);
  (void)hipMemcpy(dX, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dF, hF.data(), hF.size() * 8, hipMemcpyHostToDevice);
  std::vector<int> gc(G), gf(R), ord(R * NB);
  for (int g = 0; g < G; g++) gc[g] = g;
  for (int r = 0; r < R; r++) gf[r] = r % B;
  const bool tiled = getenv("IDENTITY") == nullptr;
  if (tiled) build_tile_order(G, B, NB, ord.data());
  else for (int r = 0; r < R * NB; r++) ord[r] = r;
  printf("order: %s\n", tiled ? "XCD tiles" : "identity");
  (void)hipMalloc(&dgc, G * 4);
  (void)hipMalloc(&dgf, R * 4);
  (void)hipMalloc(&dord, R * NB * 4);
  (void)hipMemcpy(dgc, gc.data(), G * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dgf, gf.data(), R * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dord, ord.data(), R * NB * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&drows, R * NB * sizeof(gnsscorr_acq_row));
  (void)hipMalloc(&dst, (size_t)R * NB * 16 * 8);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dst, sizeof(dst));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int it = 0; it < 3; it++) {
    if (it == 2) (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((acq_corr_kernel<0, false>), dim3(R * NB), dim3(kThreads), 0, 0, dX, dF, NB, dgc,
                       dgf, B, 16, drows, (float*)nullptr, -1, dord);
  }
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("stamped kernel: %.1f us (do not quote; stamps serialise)\n", ms * 1e3);
  std::vector<unsigned long long> st((size_t)R * NB * 16);
  (void)hipMemcpy(st.data(), dst, st.size() * 8, hipMemcpyDeviceToHost);
  const char* names[6] = {"load+mul+pass16", "pass33", "pass31+power", "argmax reduce",
                          "second-peak reduce", "next block start"};
  // one (row, block) unit per workgroup: phases 0..5 (stamps 0..5)
  double tot[6] = {0};
  const int U = R * NB;
  for (int u = 0; u < U; u++)
    for (int i = 0; i < 5; i++) tot[i] += (double)(st[u * 16 + i + 1] - st[u * 16 + i]);
  double all = 0;
  for (int i = 0; i < 5; i++) all += tot[i];
  for (int i = 0; i < 5; i++)
    printf("%-20s %8.0f cycles  %5.1f%%\n", names[i], tot[i] / U, 100.0 * tot[i] / all);
  printf("per-WG total %.0f cycles (s_memtime units)\n", all / U);
  double pro = 0, epi = 0, life = 0;
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int u = 0; u < U; u++) {
    pro += (double)(st[u * 16 + 0] - st[u * 16 + 12]);
    epi += (double)(st[u * 16 + 13] - st[u * 16 + 5]);
    life += (double)(st[u * 16 + 13] - st[u * 16 + 12]);
    if (st[u * 16 + 12] < t0) t0 = st[u * 16 + 12];
    if (st[u * 16 + 13] > t1) t1 = st[u * 16 + 13];
  }
  printf("prologue %.0f  epilogue %.0f  lifetime %.0f cycles per WG\n", pro / U, epi / U, life / U);
  printf("kernel span %.0f cycles; sum(lifetimes)/256 CUs = %.0f cycles\n", (double)(t1 - t0),
         life / 256.0);
  return 0;
}
