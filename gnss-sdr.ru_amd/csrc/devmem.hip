// devmem.hip -- device buffers, copies, events and a device-side synthetic IF
// filler, so C hosts (and bench.py) can keep IF, commands and results resident
// in HBM without any other GPU runtime in the process.
#include <dlfcn.h>
#include <stdio.h>
#include <hip/hip_runtime.h>
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

extern "C" int gnsscorr_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 13) return GNSSCORR_EINVAL;
  HIP_TRY(hipDeviceGetPCIBusId(buf, len, device));
  return GNSSCORR_OK;
}

// The HIP runtime this library's calls actually bind to: dladdr of the
// hipMalloc the library resolved (it is linked -z now, so every HIP symbol is
// bound when the library is loaded, before another copy of the runtime -- e.g.
// torch's -- can enter the global scope), and that runtime's version.
extern "C" int gnsscorr_hip_runtime(char* path, int len, int* version) {
  if (!path || len < 2 || !version) return GNSSCORR_EINVAL;
  Dl_info info = {};
  hipError_t (*const fn)(void**, size_t) = &hipMalloc;
  if (!dladdr(reinterpret_cast<void*>(fn), &info) || !info.dli_fname) {
    gnsscorr_set_error("gnsscorr_hip_runtime: dladdr(hipMalloc) failed");
    return GNSSCORR_EDEVICE;
  }
  snprintf(path, (size_t)len, "%s", info.dli_fname);
  HIP_TRY(hipRuntimeGetVersion(version));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_dev_alloc(int device, size_t bytes, void** d_ptr) {
  if (!d_ptr || bytes == 0) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipMalloc(d_ptr, bytes));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_dev_free(int device, void* d_ptr) {
  if (!d_ptr) return GNSSCORR_OK;
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipFree(d_ptr));
  return GNSSCORR_OK;
}

// The plain copies wait for the whole device first: a hipMemcpy on the null
// stream is not ordered against the contexts' non-blocking streams, so a
// copy issued while a kernel still uses the buffer would race with it.
extern "C" int gnsscorr_memcpy_htod(int device, void* d, const void* h, size_t bytes) {
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_memcpy_dtoh(int device, void* h, const void* d, size_t bytes) {
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_dev_synchronize(int device) {
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_event_create(int device, void** ev) {
  if (!ev) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(device));
  hipEvent_t e;
  HIP_TRY(hipEventCreate(&e));
  *ev = (void*)e;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_event_record(void* ev, void* stream) {
  HIP_TRY(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_stream_wait_event(void* stream, void* ev) {
  if (!ev) return GNSSCORR_EINVAL;
  HIP_TRY(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_event_elapsed_ms(void* start, void* stop, float* ms) {
  if (!ms) return GNSSCORR_EINVAL;
  HIP_TRY(hipEventSynchronize((hipEvent_t)stop));
  HIP_TRY(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_event_destroy(void* ev) {
  if (ev) HIP_TRY(hipEventDestroy((hipEvent_t)ev));
  return GNSSCORR_OK;
}

namespace {
// splitmix64 hash -> four 2-bit levels {-3,-1,1,3} per 32-bit draw
__global__ void fill_if2_kernel(int8_t* __restrict__ d, size_t n, uint64_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t base = i * 8;
  if (base >= n) return;
  uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (base + k < n) {
      const int v = (int)((z >> (2 * k)) & 3u);
      d[base + k] = (int8_t)(2 * v - 3);
    }
  }
}
}  // namespace

extern "C" int gnsscorr_dev_fill_if2(int device, int8_t* d, size_t bytes, uint64_t seed) {
  if (!d || !bytes) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(device));
  const size_t threads = (bytes + 7) / 8;
  hipLaunchKernelGGL(fill_if2_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, 0, d,
                     bytes, seed);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  return GNSSCORR_OK;
}
