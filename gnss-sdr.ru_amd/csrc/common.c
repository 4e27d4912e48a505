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
const char *gnsscorr_version(void) { return "gnsscorr 0.1.0 (gfx950)"; }
