/* common.c -- error reporting and version for the C ABI. */
#include "gnsscorr_internal.h"
#include <stdarg.h>
#include <stdio.h>

static __thread char g_err[512];

void gnsscorr_set_error(const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}

const char *gnsscorr_last_error(void) { return g_err; }
const char *gnsscorr_version(void) { return "gnsscorr 0.2.0 (gfx950)"; }

/* GNSSCORR_IF_PACKED2 packing (gnsscorr.h): level 2c-3 -> code c, element e in
 * bits 2*(e%4) of byte e/4 (the GN3S LUT, gps_source.cpp:692, inverted). */
int gnsscorr_pack2(const int8_t *in, int64_t n, uint8_t *out)
{
  if (!in || !out || n < 0) {
    gnsscorr_set_error("gnsscorr_pack2: bad arguments");
    return GNSSCORR_EINVAL;
  }
  for (int64_t e = 0; e < n; e++) {
    const int v = in[e];
    if (v != -3 && v != -1 && v != 1 && v != 3) {
      gnsscorr_set_error("gnsscorr_pack2: element %lld = %d is not a 2-bit level", (long long)e, v);
      return GNSSCORR_EINVAL;
    }
  }
  for (int64_t b = 0; b < (n + 3) / 4; b++) {
    unsigned byte = 0;
    for (int j = 0; j < 4 && 4 * b + j < n; j++) byte |= (unsigned)((in[4 * b + j] + 3) >> 1) << (2 * j);
    out[b] = (uint8_t)byte;
  }
  return GNSSCORR_OK;
}
