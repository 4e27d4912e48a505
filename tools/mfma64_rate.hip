// Throughput probe: fp64 MFMA (v_mfma_f64_16x16x4_f64) alone, fp64 VALU FMA
// alone, and both at once on the same SIMDs (waves 0-3 matrix, 4-7 vector);
// probe32 the same for fp32 (v_mfma_f32_16x16x4_f32 beside packed v_pk_fma_f32).
// Decides whether the radix-31 stage of acq64_corr_kernel gains from moving
// its real 16x16 coefficient products onto the matrix pipe.
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma64_rate.hip -o tools/mfma64_rate
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double v4d __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

// mode bit 0: waves 0-3 run MFMA chains; bit 1: waves 4-7 run VALU chains
__global__ __launch_bounds__(512) void probe(double* out, int mode, double seed) {
  const int w = threadIdx.x >> 6;
  double acc = 0.0;
  if (w < 4 && (mode & 1)) {
    v4d c0 = {seed, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = seed + threadIdx.x, b = 1.0 - seed;
    for (int i = 0; i < kIters; i++) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
    acc = c0.x + c1.y + c2.z + c3.w;
  }
  if (w >= 4 && (mode & 2)) {
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = seed + k + threadIdx.x;
    const double m = 1.0 - 1e-9 * seed, d = 1e-12;
    // 4 * kIters * 8 FMAs per lane = the same flops per wave as the MFMA loop
    // would need 16x16x4x2 / 64 / 2 = 16 FMAs per MFMA: 4 chains x 16 = 64 per iter
    for (int i = 0; i < kIters; i++) {
#pragma unroll
      for (int r = 0; r < 8; r++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = fma(x[k], m, d);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) acc += x[k];
  }
  if (acc == 12345.678) out[blockIdx.x] = acc;
}

// fp32: mode bit 0 MFMA (waves 0-3), bit 1 packed fp32 FMA (waves 4-7)
__global__ __launch_bounds__(512) void probe32(double* out, int mode, float seed) {
  const int w = threadIdx.x >> 6;
  float acc = 0.f;
  if (w < 4 && (mode & 1)) {
    v4f c0 = {seed, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    float a = seed + threadIdx.x, b = 1.f - seed;
    for (int i = 0; i < kIters; i++) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
    acc = c0.x + c1.y + c2.z + c3.w;
  }
  if (w >= 4 && (mode & 2)) {
    v2f x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = (v2f){seed + k + threadIdx.x, seed - k};
    const v2f m = {1.f - 1e-6f * seed, 1.f - 1e-6f * seed}, d = {1e-7f, 1e-7f};
    for (int i = 0; i < kIters; i++) {
#pragma unroll
      for (int r = 0; r < 8; r++)
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = __builtin_elementwise_fma(x[k], m, d);
    }
#pragma unroll
    for (int k = 0; k < 8; k++) acc += x[k].x + x[k].y;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;
}

int main() {
  double* out;
  hipMalloc(&out, 1 << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = 256 * 4;
  const char* names[] = {"", "mfma only", "valu only", "mfma + valu"};
  for (int rep = 0; rep < 2; rep++)
    for (int mode = 1; mode <= 3; mode++) {
      probe<<<grid, 512>>>(out, mode, 0.5);
      hipEventRecord(e0);
      probe<<<grid, 512>>>(out, mode, 0.5);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double mf = (mode & 1) ? (double)grid * 4 * kIters * 4 * 2048 : 0;
      const double vf = (mode & 2) ? (double)grid * 4 * 64 * kIters * 64 * 2 : 0;
      printf("%-12s %8.3f ms  mfma %6.1f TF  valu %6.1f TF  total %6.1f TF\n", names[mode], ms,
             mf / ms * 1e-9, vf / ms * 1e-9, (mf + vf) / ms * 1e-9);
    }
  for (int rep = 0; rep < 2; rep++)
    for (int mode = 1; mode <= 3; mode++) {
      probe32<<<grid, 512>>>(out, mode, 0.5f);
      hipEventRecord(e0);
      probe32<<<grid, 512>>>(out, mode, 0.5f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // 16x16x4 f32: 2048 flop; VALU: 64 packed FMAs x 2 lanes x 2 flop per iteration
      const double mf = (mode & 1) ? (double)grid * 4 * kIters * 4 * 2048 : 0;
      const double vf = (mode & 2) ? (double)grid * 4 * 64 * kIters * 64 * 4 : 0;
      printf("f32 %-12s %8.3f ms  mfma %6.1f TF  valu %6.1f TF  total %6.1f TF\n", names[mode], ms,
             mf / ms * 1e-9, vf / ms * 1e-9, (mf + vf) / ms * 1e-9);
    }
  return 0;
}
