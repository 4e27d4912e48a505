// sdr_frontend.hip -- GPS-SDR sample front end on gfx950.
//
// Reference: REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/
//   objects/gps_source.cpp:684-767  GPS_Source::Read_GN3S -- per 5-ms block of
//       20000 2-bit samples: LUT {-3,-1,1,3}, mix by a 1024-entry table NCO
//       (uint32 phase, index phase >> 22, step 2557223528; tables +-8 cos/sin,
//       :92-96), double products truncated to int16
//   objects/gps_source.cpp:933-943  Resample_GN3S -- out[i] = in[gdec[i]],
//       gdec[i] = floor((i+1)*4000/2048) (:433-437), 10240 outputs = 5 packets
//   accessories/misc.cpp:174-197    downsample -- keep sample lcv when the
//       uint32 phase accumulator (step floor(2^32 fdest/fsource)) wraps
//
// The sequential loops become closed forms, so every output sample is one
// independent thread:
//   GN3S:  input n = ((i+1)*125) >> 6 of block b, phase = phase0 + (b*20000+n)*step
//          (mod 2^32); the int16 products are a host-built 4 x 1024 table
//          (gnsscorr_sdr_gn3s_products), bit-exact with the double arithmetic.
//          Output 10239 of every block reads in[20000], one past the 20000
//          samples the reference just wrote (its buff[40932] member keeps that
//          entry at its initial zero), so it is (0, 0).
//   downsample: output k >= 1 is input ceil(k*2^32/step), output 0 is input 0.
// Input formats: 1 sample per byte (the reference's gbuff, low 2 bits used) or
// packed 4 samples per byte (sample j of a byte in bits 2j..2j+1) -- 4x fewer
// bytes over PCIe and from HBM.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include "gnsscorr_internal.h"

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      gnsscorr_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                     \
      return GNSSCORR_EDEVICE;                                                          \
    }                                                                                   \
  } while (0)

namespace {

constexpr int kBlkIn = GNSSCORR_GN3S_BLOCK_IN;     // 20000 samples per 5 ms
constexpr int kBlkOut = GNSSCORR_GN3S_BLOCK_OUT;   // 10240 = 5 x 2048
constexpr int kThreads = 256;

// out[b][i] (int16 I, Q packed in one uint32, I in the low half like CPX).
// A thread writes four consecutive outputs of one block as one 16-byte store.
// The product lookups are random in the 1024-entry phase, so the table sits in
// LDS (an L1 gather touches one cache line per lane).  Only codes 2, 3 (LUT
// +1, +3) are staged: (int16)(-x) == -(int16)(x) for the truncating cast, so
// codes 1, 0 are their packed negations (exact).  grid = (kBlkOut / 4 /
// kThreads) x min(n_blocks, kGridY); each workgroup loops over blocks b =
// blockIdx.y + k * gridDim.y, amortising the 8 KiB staging.
constexpr int kQuads = kBlkOut / 4;   // 2560 16-byte stores per block
constexpr int kGridY = 192;           // 10 x 192 workgroups: ~8 per CU

typedef short short2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t gn3s_sample(const uint8_t* __restrict__ in, int fmt, uint32_t s0,
                                                int i, uint32_t phase0, uint32_t step,
                                                const uint32_t* tab) {
  const int n = ((i + 1) * 125) >> 6;   // floor((i+1)*4000/2048)
  if (n >= kBlkIn) return 0u;           // output 10239 reads the zero past the block
  const uint32_t s = s0 + (uint32_t)n;  // < 2^31 (checked on the host)
  const uint32_t code = fmt == 0 ? (in[s] & 3u) : ((in[s >> 2] >> (2 * (s & 3))) & 3u);
  const uint32_t ph = phase0 + s * step;
  const uint32_t v = tab[((code >= 2 ? code : 3u - code) - 2u) * 1024 + (ph >> 22)];
  if (code >= 2) return v;
  const short2_t neg = -__builtin_bit_cast(short2_t, v);
  return __builtin_bit_cast(uint32_t, neg);
}

__global__ __launch_bounds__(kThreads) void gn3s_kernel(const uint8_t* __restrict__ in, int fmt,
                                                        int n_blocks, uint32_t phase0,
                                                        uint32_t step,
                                                        const uint32_t* __restrict__ prod,
                                                        uint32_t* __restrict__ out) {
  __shared__ uint32_t tab[2 * 1024];
  for (int k = threadIdx.x; k < 2 * 1024; k += kThreads) tab[k] = prod[2 * 1024 + k];
  __syncthreads();
  const int q = blockIdx.x * kThreads + threadIdx.x;   // < kQuads: the grid is exact
  for (int b = blockIdx.y; b < n_blocks; b += gridDim.y) {
    const int i = 4 * q;
    const uint32_t s0 = (uint32_t)b * kBlkIn;
    uint4 v;
    v.x = gn3s_sample(in, fmt, s0, i, phase0, step, tab);
    v.y = gn3s_sample(in, fmt, s0, i + 1, phase0, step, tab);
    v.z = gn3s_sample(in, fmt, s0, i + 2, phase0, step, tab);
    v.w = gn3s_sample(in, fmt, s0, i + 3, phase0, step, tab);
    *reinterpret_cast<uint4*>(out + (size_t)b * kBlkOut + i) = v;
  }
}

__global__ __launch_bounds__(kThreads) void downsample_kernel(const uint32_t* __restrict__ src,
                                                              int n_out, uint32_t step,
                                                              uint32_t* __restrict__ dst) {
  const int k = blockIdx.x * kThreads + threadIdx.x;
  if (k >= n_out) return;
  // smallest lcv with lcv * step >= k * 2^32 (the k-th wrap); k = 0 -> 0
  const unsigned long long num = ((unsigned long long)k << 32) + step - 1;
  dst[k] = src[num / step];
}

}  // namespace

struct gnsscorr_sdr_fe_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t* d_prod = nullptr;   // 4 x 1024 (I | Q << 16)
  uint8_t* d_in = nullptr;      // host-API staging
  uint32_t* d_out = nullptr;
  size_t cap_in = 0, cap_out = 0;
};

extern "C" int gnsscorr_sdr_fe_create(gnsscorr_sdr_fe_ctx** out, int device) {
  if (!out) {
    gnsscorr_set_error("gnsscorr_sdr_fe_create: null out");
    return GNSSCORR_EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gnsscorr_set_error("gnsscorr_sdr_fe_create: no HIP device");
    return GNSSCORR_ENODEV;
  }
  if (device < 0 || device >= ndev) {
    gnsscorr_set_error("gnsscorr_sdr_fe_create: device %d out of range", device);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(device));
  auto* c = new gnsscorr_sdr_fe_ctx();
  c->device = device;
  int16_t prod[4 * 1024 * 2];
  gnsscorr_sdr_gn3s_products(prod);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_prod, sizeof(prod)) != hipSuccess ||
      hipMemcpy(c->d_prod, prod, sizeof(prod), hipMemcpyHostToDevice) != hipSuccess) {
    gnsscorr_sdr_fe_destroy(c);
    gnsscorr_set_error("gnsscorr_sdr_fe_create: device allocation failed");
    return GNSSCORR_ENOMEM;
  }
  *out = c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_fe_destroy(gnsscorr_sdr_fe_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->d_prod) (void)hipFree(c->d_prod);
  if (c->d_in) (void)hipFree(c->d_in);
  if (c->d_out) (void)hipFree(c->d_out);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GNSSCORR_OK;
}

static size_t gn3s_in_bytes(int fmt, int n_blocks) {
  return fmt == 0 ? (size_t)n_blocks * kBlkIn : (size_t)n_blocks * (kBlkIn / 4);
}

extern "C" int gnsscorr_sdr_gn3s_dev(gnsscorr_sdr_fe_ctx* c, const uint8_t* d_in, int fmt,
                                     int n_blocks, uint32_t* phase, uint32_t step,
                                     int16_t* d_out) {
  if (!c || !d_in || !d_out || !phase || (fmt != 0 && fmt != 1) || n_blocks < 1 ||
      (long)n_blocks * kBlkIn >= (1L << 31)) {
    gnsscorr_set_error("gnsscorr_sdr_gn3s: bad arguments (fmt %d, blocks %d)", fmt, n_blocks);
    return GNSSCORR_EINVAL;
  }
  if ((uintptr_t)d_out & 15u) {
    gnsscorr_set_error("gnsscorr_sdr_gn3s_dev: d_out must be 16-byte aligned");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->device));
  static_assert(kQuads % kThreads == 0, "exact grid of 16-byte output stores");
  hipLaunchKernelGGL(gn3s_kernel, dim3(kQuads / kThreads,
                                       (unsigned)(n_blocks < kGridY ? n_blocks : kGridY)),
                     dim3(kThreads), 0, c->stream, d_in, fmt, n_blocks, *phase, step, c->d_prod,
                     (uint32_t*)d_out);
  HIP_TRY(hipGetLastError());
  *phase += (uint32_t)((uint64_t)n_blocks * kBlkIn * step);   // the NCO runs over every input
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_gn3s(gnsscorr_sdr_fe_ctx* c, const uint8_t* h_in, int fmt,
                                 int n_blocks, uint32_t* phase, uint32_t step, int16_t* h_out) {
  if (!c || !h_in || !h_out || n_blocks < 1) {
    gnsscorr_set_error("gnsscorr_sdr_gn3s: bad arguments");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->device));
  const size_t nb = gn3s_in_bytes(fmt, n_blocks);
  const size_t no = (size_t)n_blocks * kBlkOut * 4;
  if (nb > c->cap_in) {
    if (c->d_in) (void)hipFree(c->d_in);
    c->d_in = nullptr;
    c->cap_in = 0;
    HIP_TRY(hipMalloc(&c->d_in, nb));
    c->cap_in = nb;
  }
  if (no > c->cap_out) {
    if (c->d_out) (void)hipFree(c->d_out);
    c->d_out = nullptr;
    c->cap_out = 0;
    HIP_TRY(hipMalloc(&c->d_out, no));
    c->cap_out = no;
  }
  HIP_TRY(hipMemcpyAsync(c->d_in, h_in, nb, hipMemcpyHostToDevice, c->stream));
  const int rc = gnsscorr_sdr_gn3s_dev(c, c->d_in, fmt, n_blocks, phase, step, (int16_t*)c->d_out);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(h_out, c->d_out, no, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

// number of samples downsample() keeps from n_src inputs (0 if n_src < 1)
extern "C" int gnsscorr_sdr_downsample_count(int n_src, double f_dest, double f_source,
                                             uint32_t* step_out) {
  if (n_src < 1 || !(f_dest > 0) || !(f_dest < f_source)) return 0;
  const uint32_t step = (uint32_t)floor(4294967296.0 * f_dest / f_source);
  if (step_out) *step_out = step;
  if (step == 0) return 1;
  return 1 + (int)(((unsigned long long)(n_src - 1) * step) >> 32);
}

extern "C" int gnsscorr_sdr_downsample_dev(gnsscorr_sdr_fe_ctx* c, const int16_t* d_src,
                                           int n_src, double f_dest, double f_source,
                                           int16_t* d_dest, int* n_out) {
  uint32_t step = 0;
  const int k = gnsscorr_sdr_downsample_count(n_src, f_dest, f_source, &step);
  if (!c || !d_src || !d_dest || k < 1 || step == 0) {
    gnsscorr_set_error("gnsscorr_sdr_downsample: bad arguments (n %d, fdest %g, fsource %g)",
                       n_src, f_dest, f_source);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->device));
  hipLaunchKernelGGL(downsample_kernel, dim3((k + kThreads - 1) / kThreads), dim3(kThreads), 0,
                     c->stream, (const uint32_t*)d_src, k, step, (uint32_t*)d_dest);
  HIP_TRY(hipGetLastError());
  if (n_out) *n_out = k;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sdr_fe_sync(gnsscorr_sdr_fe_ctx* c) {
  if (!c) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" void* gnsscorr_sdr_fe_stream(gnsscorr_sdr_fe_ctx* c) { return c ? c->stream : nullptr; }
