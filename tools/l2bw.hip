// tools/l2bw.hip -- L2 -> CU read bandwidth for the acquisition correlation
// kernel's access pattern (each unit reads one X row and one F row of 16
// planes x 1024 complex fp32 with 16-byte loads, XCD-tiled unit order).
// Variants: threads per workgroup, LDS reservation (1 or many workgroups per
// CU), loads in flight per thread.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
constexpr int NPAD = 16 * 1024;
typedef float f4v __attribute__((ext_vector_type(4)));

template <int T, int LDSB, int GROUP>
__global__ __launch_bounds__(T) void rd(const float2* X, const float2* F, int n_bins, int n_units,
                                         float* out) {
  __shared__ float pad[LDSB / 4];
  const int u = blockIdx.x;
  const int row = u / 2, blk = u % 2;
  const int g = row / n_bins, bin = row % n_bins;
  const auto rx = __builtin_amdgcn_make_buffer_rsrc((void*)(X + (long)((bin % 2) * 2 + blk) * NPAD), 0, NPAD * 8, 0x00020000);
  const auto rf = __builtin_amdgcn_make_buffer_rsrc((void*)(F + (long)g * NPAD), 0, NPAD * 8, 0x00020000);
  f4v acc = {0, 0, 0, 0};
  constexpr int COLS = 1024 / (2 * T) > 0 ? 1024 / (2 * T) : 1;   // 2-column chunks per thread
  for (int c = 0; c < COLS; c++) {
    const int voff = (threadIdx.x + c * T) * 16;
#pragma unroll
    for (int a0 = 0; a0 < 16; a0 += GROUP) {
      f4v xs[GROUP], fs[GROUP];
#pragma unroll
      for (int a = 0; a < GROUP; a++) {
        xs[a] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rx, voff, (a0 + a) * 8192, 0));
        fs[a] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(rf, voff, (a0 + a) * 8192, 0));
      }
#pragma unroll
      for (int a = 0; a < GROUP; a++) acc += xs[a] * fs[a];
    }
  }
  if (LDSB > 16) pad[threadIdx.x % (LDSB / 4)] = acc.x;
  __syncthreads();
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[u] = pad[0];
}

template <int T, int LDSB, int GROUP>
void run(const float2* dX, const float2* dF, float* dout, int B, int U) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e9f;
  for (int it = 0; it < 10; it++) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((rd<T, LDSB, GROUP>), dim3(U), dim3(T), 0, 0, dX, dF, B, U, dout);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (it > 1 && ms < best) best = ms;
  }
  const double bytes = (double)U * 2 * NPAD * 8;
  printf("T=%4d lds=%6d group=%2d: %7.1f us  %6.2f TB/s\n", T, LDSB, GROUP, best * 1e3, bytes / (best * 1e-3) / 1e12);
}

int main() {
  const int G = 32, B = 41, U = G * B * 2;
  float2 *dX, *dF;
  float* dout;
  (void)hipMalloc(&dX, (size_t)B * 2 * NPAD * 8);
  (void)hipMalloc(&dF, (size_t)G * NPAD * 8);
  (void)hipMemset(dX, 0, (size_t)B * 2 * NPAD * 8);
  (void)hipMemset(dF, 0, (size_t)G * NPAD * 8);
  (void)hipMalloc(&dout, U * 4);
  run<512, 131072, 16>(dX, dF, dout, B, U);
  run<512, 131072, 8>(dX, dF, dout, B, U);
  run<512, 131072, 4>(dX, dF, dout, B, U);
  run<512, 16, 16>(dX, dF, dout, B, U);
  run<512, 16, 8>(dX, dF, dout, B, U);
  run<1024, 131072, 8>(dX, dF, dout, B, U);
  run<256, 16, 16>(dX, dF, dout, B, U);
  run<256, 16, 4>(dX, dF, dout, B, U);
  return 0;
}
