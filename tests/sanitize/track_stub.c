/* tests/sanitize/track_stub.c -- TEST SCAFFOLDING for the host-only sanitizer
 * build (tests/test_sanitize_host.py): a deterministic host stand-in for the
 * four tracking-context calls the OSG shim (csrc/osg_legacy.c) makes, so the
 * shim's REG_read/REG_write bookkeeping runs under ASan/UBSan without a GPU.
 * It is never linked into libgnsscorr.so. */
#include <stdlib.h>
#include <string.h>
#include "gnsscorr.h"

struct gnsscorr_track_ctx { int n; int calls; gnsscorr_chan_state st[14]; };

int gnsscorr_track_create(gnsscorr_track_ctx **out, const gnsscorr_track_cfg *cfg)
{
  if (!out || !cfg || cfg->n_channels < 1 || cfg->n_channels > 14) return GNSSCORR_EINVAL;
  *out = calloc(1, sizeof(gnsscorr_track_ctx));
  (*out)->n = cfg->n_channels;
  return GNSSCORR_OK;
}
int gnsscorr_track_destroy(gnsscorr_track_ctx *c) { free(c); return GNSSCORR_OK; }
int gnsscorr_track_get_state(gnsscorr_track_ctx *c, gnsscorr_chan_state *s)
{
  memcpy(s, c->st, sizeof(gnsscorr_chan_state) * c->n);
  return GNSSCORR_OK;
}
int gnsscorr_track_set_state(gnsscorr_track_ctx *c, const gnsscorr_chan_state *s)
{
  memcpy(c->st, s, sizeof(gnsscorr_chan_state) * c->n);
  return GNSSCORR_OK;
}
/* dumps on every other call for odd channels; sums derived from the IF bytes */
int gnsscorr_track(gnsscorr_track_ctx *c, const int8_t *h_if, int64_t stride, int n_streams,
                   int64_t nsamp, const gnsscorr_nco_cmd *cmds, gnsscorr_track_result *res,
                   int32_t *all_dumps, int *tic)
{
  (void)stride; (void)n_streams; (void)all_dumps;
  long sum = 0;
  for (int64_t i = 0; i < 2 * nsamp; i++) sum += h_if[i];
  for (int ch = 0; ch < c->n; ch++) {
    memset(&res[ch], 0, sizeof res[ch]);
    if ((ch & 1) && (c->calls & 1)) {
      res[ch].n_dumps = 1;
      for (int k = 0; k < 6; k++) res[ch].dump[k] = (int32_t)(sum + cmds[ch].prn * 7 + k);
    }
    res[ch].msbit_reg = c->calls + ch;
    c->st[ch].ms_counter = c->calls;
  }
  c->calls++;
  if (tic) *tic = (c->calls % 5) == 0;
  return GNSSCORR_OK;
}
