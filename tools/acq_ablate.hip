// tools/acq_ablate.hip -- diagnostic: time the acquisition correlation kernel
// with phases removed (ACQ_SKIP, see acq.hip) on config-2-shaped synthetic
// spectra.  Build one binary per ACQ_SKIP value on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DACQ_SKIP=<k> -Iinclude \
//         -Ignss-sdr.ru_amd/csrc tools/acq_ablate.hip build/common.c.o -o /tmp/ab<k>
// Prints the mean kernel time (us) for unshifted and shifted spectrum reads.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include "../gnss-sdr.ru_amd/csrc/acq.hip"

int main() {
  const int G = 32, B = 41, R = G * B, NB = 2;
  std::vector<float2> hX((size_t)B * NB * NPAD), hF((size_t)G * NPAD);
  srand(1);
  for (auto& v : hX) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  for (auto& v : hF) v = make_float2(rand() / (float)RAND_MAX - 0.5f, rand() / (float)RAND_MAX - 0.5f);
  float2 *dX, *dF;
  int *dgc, *dgf, *dord;
  int4* dfm;
  gnsscorr_acq_row* drows;
  (void)hipMalloc(&dX, hX.size() * 8);
  (void)hipMalloc(&dF, hF.size() * 8);
  (void)hipMemcpy(dX, hX.data(), hX.size() * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(dF, hF.data(), hF.size() * 8, hipMemcpyHostToDevice);
  std::vector<int> gc(G), gf(R), ord(R * NB);
  for (int g = 0; g < G; g++) gc[g] = g;
  for (int r = 0; r < R; r++) gf[r] = r % B;
  build_tile_order(G, B, NB, ord.data());
  (void)hipMalloc(&dgc, G * 4);
  (void)hipMalloc(&dgf, R * 4);
  (void)hipMalloc(&dord, R * NB * 4);
  (void)hipMalloc(&dfm, B * sizeof(int4));
  (void)hipMemcpy(dgc, gc.data(), G * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dgf, gf.data(), R * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dord, ord.data(), R * NB * 4, hipMemcpyHostToDevice);
  (void)hipMalloc(&drows, R * NB * sizeof(gnsscorr_acq_row));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int shifted = 0; shifted < 2; shifted++) {
    std::vector<int4> fm(B);
    for (int b = 0; b < B; b++) {
      const int m = (b - 20 + N) % N;
      fm[b] = shifted ? make_int4(b & 1, (15 * m) & 15, (2 * m) % 3, ((4 * m) % 11) * 32 + m % 31)
                      : make_int4(b, 0, 0, 0);
    }
    (void)hipMemcpy(dfm, fm.data(), B * sizeof(int4), hipMemcpyHostToDevice);
    float best = 1e9f;
    for (int it = 0; it < 12; it++) {
      (void)hipEventRecord(e0, 0);
#ifdef PIPE
      hipLaunchKernelGGL(acq_corr_pipe_kernel, dim3(256), dim3(kPipeThreads), 0, 0, dX, dF, NB, dgc,
                         dgf, B, 16, drows, dord, dfm, R * NB);
#else
      hipLaunchKernelGGL((acq_corr_kernel<0, false>), dim3(R * NB), dim3(kThreads), 0, 0, dX, dF,
                         NB, dgc, dgf, B, 16, drows, (float*)nullptr, -1, dord, dfm);
#endif
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it >= 2 && ms < best) best = ms;
    }
#ifdef PIPE
    const char* kern = "pipe";
#else
    const char* kern = "old";
#endif
    printf("%s plane=%d ACQ_SKIP=%d %s: %.1f us\n", kern, kPlane, ACQ_SKIP, shifted ? "shifted" : "aligned", best * 1e3);
  }
  return 0;
}
