// tools/trk_slots_mb.hip -- does a second LDS-DMA piece slot per wave pay at the
// tracking kernel's shape?  Microbenchmark of osg_stream_kernel's memory pattern
// (diagnostic only): 12288 waves (4 per SIMD, 4 per workgroup), each streaming its
// own IF (C_s = 1) or one of 1024 streams shared by 12 waves (receiver layout,
// L2-resident) in 4 KiB pieces by global_load_lds_dwordx4, with ~400 VALU
// instructions of dot4 work per piece on the piece's 64 bytes per lane (the real
// kernel's per-piece VALU count).  SLOTS pieces in flight; the slot read is inline
// asm so the compiler does not drain the other slot's DMA before it; the LDS per
// wave is padded to the real kernel's (1 slot: 7.9 KiB; 2 slots: 8.4 KiB) so 16
// waves share a CU either way.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kPiece = 4096;   // bytes per wave per piece
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int SLOTS, int WAVE_LDS, int WORK>
__global__ __launch_bounds__(256, 4) void mb(const int8_t* __restrict__ buf, long stream_bytes,
                                             int n_pieces, int shared, int* out) {
  extern __shared__ uint4 s_dyn[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + wave;
  const int stream = shared ? (w / 12) : w;
  const int8_t* src = buf + (long)stream * stream_bytes;
  uint4* slot0 = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(s_dyn) + wave * WAVE_LDS);
  auto issue = [&](int p) {
    uint4* slot = slot0 + (p % SLOTS) * (kPiece / 16);
    const int8_t* g = src + (long)p * kPiece;
#pragma unroll
    for (int r = 0; r < 4; r++)
      __builtin_amdgcn_global_load_lds((const void*)(g + 16 * (r * 64 + lane)),
                                       (__attribute__((address_space(3))) void*)(slot + r * 64), 16,
                                       0, 0);
  };
  for (int p = 0; p < SLOTS && p < n_pieces; p++) issue(p);
  uint32_t acc0 = lane, acc1 = 1, acc2 = 2, acc3 = 3;
  for (int p = 0; p < n_pieces; p++) {
    if (SLOTS == 2 && p + 1 < n_pieces) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint4*)(
        slot0 + (p % SLOTS) * (kPiece / 16) + 4 * lane);
    u32x4 v0, v1, v2, v3;
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\t"
        "ds_read_b128 %2, %4 offset:32\n\tds_read_b128 %3, %4 offset:48\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
        : "v"(la)
        : "memory");
    if (p + SLOTS < n_pieces) issue(p + SLOTS);
    const uint32_t x[16] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w,
                            v2.x, v2.y, v2.z, v2.w, v3.x, v3.y, v3.z, v3.w};
#pragma unroll
    for (int k = 0; k < WORK; k++) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        acc0 = __builtin_amdgcn_sdot4((int)x[i], (int)acc1, (int)acc0, false);
        acc1 = __builtin_amdgcn_sdot4((int)x[i], (int)acc2, (int)acc1, false);
        acc2 = __builtin_amdgcn_sdot4((int)x[i], (int)acc3, (int)acc2, false);
        acc3 = __builtin_amdgcn_sdot4((int)x[i], (int)acc0, (int)acc3, false);
      }
    }
  }
  if ((acc0 ^ acc1 ^ acc2 ^ acc3) == 0x12345u) out[w] = 1;
}

template <int SLOTS, int WAVE_LDS, int WORK>
float run(const int8_t* buf, long sb, int n_pieces, int shared, int* out, int waves) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const size_t lds = 4 * WAVE_LDS;
  for (int i = 0; i < 2; i++)
    hipLaunchKernelGGL((mb<SLOTS, WAVE_LDS, WORK>), dim3(waves / 4), dim3(256), lds, 0, buf, sb,
                       n_pieces, shared, out);
  hipEventRecord(a);
  const int reps = 5;
  for (int i = 0; i < reps; i++)
    hipLaunchKernelGGL((mb<SLOTS, WAVE_LDS, WORK>), dim3(waves / 4), dim3(256), lds, 0, buf, sb,
                       n_pieces, shared, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main() {
  const int waves = 12288, n_pieces = 80;   // 10 calls of 8 pieces
  const long sb = (long)n_pieces * kPiece;
  int8_t* buf;
  int* out;
  if (hipMalloc(&buf, sb * waves) != hipSuccess || hipMalloc(&out, waves * 4) != hipSuccess) {
    printf("alloc failed\n");
    return 1;
  }
  hipMemset(buf, 1, sb * waves);
  const double bytes = (double)sb * waves;
  for (int shared = 0; shared < 2; shared++) {
    const char* lay = shared ? "rx12 (L2)" : "cs1 (HBM)";
    float t1 = run<1, 7936, 6>(buf, sb, n_pieces, shared, out, waves);
    float t2 = run<2, 8448, 6>(buf, sb, n_pieces, shared, out, waves);
    float t1l = run<1, 7936, 3>(buf, sb, n_pieces, shared, out, waves);
    float t2l = run<2, 8448, 3>(buf, sb, n_pieces, shared, out, waves);
    float t0 = run<1, 7936, 0>(buf, sb, n_pieces, shared, out, waves);
    float t0b = run<2, 8448, 0>(buf, sb, n_pieces, shared, out, waves);
    printf("%s: us per call (8 pieces) | work 384 VALU/piece: 1 slot %.2f, 2 slots %.2f | "
           "192: 1 slot %.2f, 2 slots %.2f | no work: 1 slot %.2f (%.2f TB/s), 2 slots %.2f "
           "(%.2f TB/s)\n",
           lay, t1 * 100, t2 * 100, t1l * 100, t2l * 100, t0 * 100,
           shared ? 0.0 : bytes / (t0 * 1e-3) / 1e12, t0b * 100,
           shared ? 0.0 : bytes / (t0b * 1e-3) / 1e12);
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}
