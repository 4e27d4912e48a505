// if2.h -- device helpers for the IF sample formats of the batched API.
//
// GNSSCORR_IF_PACKED2 (gnsscorr.h): four 2-bit codes per byte, element e of a
// stream in bits 2*(e&3)..2*(e&3)+1 of byte e>>2 (elements are I,Q,I,Q,... for
// complex streams), code c -> level 2c-3, i.e. the GN3S LUT {-3,-1,1,3} of
// GPS_Source::Read_GN3S (REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/
// objects/gps_source.cpp:692).  A packed stream holds exactly the int8 stream
// of those levels in a quarter of the bytes, so every kernel result is
// identical to the int8 path on the unpacked samples.
#ifndef GNSSCORR_IF2_H
#define GNSSCORR_IF2_H
#include <hip/hip_runtime.h>
#include <stdint.h>

// one packed byte (4 elements) -> 4 int8 levels, element j in byte j
__device__ __forceinline__ uint32_t if2_expand_byte(uint32_t b) {
  uint32_t t = b | (b << 6);    // codes 0, 1 -> bytes 0, 1 (bits 0-1, 8-9)
  t |= t << 12;                 // codes 2, 3 -> bytes 2, 3 (bits 16-17, 24-25)
  t &= 0x03030303u;
  // v_perm_b32 byte select from {0, table}: selector c picks table byte c
  return __builtin_amdgcn_perm(0u, 0x0301FFFDu, t);   // {-3, -1, 1, 3} as int8
}

// one packed 32-bit word (16 elements) -> four int8 words
__device__ __forceinline__ uint4 if2_expand_word(uint32_t p) {
  return make_uint4(if2_expand_byte(p & 0xFFu), if2_expand_byte((p >> 8) & 0xFFu),
                    if2_expand_byte((p >> 16) & 0xFFu), if2_expand_byte(p >> 24));
}

// element e of a stream (int8 or packed)
__device__ __forceinline__ int if_elem(const int8_t* __restrict__ base, int64_t e, bool packed) {
  if (packed) {
    const uint32_t b = reinterpret_cast<const uint8_t*>(base)[e >> 2];
    return 2 * (int)((b >> (2 * (e & 3))) & 3u) - 3;
  }
  return base[e];
}

// bytes holding n elements
__host__ __device__ __forceinline__ int64_t if_bytes(int64_t n_elems, bool packed) {
  return packed ? (n_elems + 3) >> 2 : n_elems;
}
#endif
