/*
 * osg_legacy.c -- the OSGPS software-correlator symbols on top of the batched
 * GPU tracking API (drop-in for osgnss_next_step/src/correlator/correlator.c).
 *
 *   correlator_init(double)          correlator.c:107-132
 *   Sim_GP2021_int(char *, long)     correlator.c:148-316
 *   int REG_read[256], REG_write[256] correlator.h:4 (register map :9-20)
 *
 * REG_write -> per-channel NCO command, one synchronous GPU call, results ->
 * REG_read latches, exactly as the reference leaves them after its loop.
 */
#include "gnsscorr.h"
#include "gnsscorr_osg.h"
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int REG_read[256], REG_write[256];

/* receiver globals written by correlator_init (globals.h:41-49) */
double Carrier_DCO_Delta, Code_DCO_Delta;
long gps_code_ref, gps_carrier_ref, glonass_code_ref, glonass_carrier_ref, d_freq;

static struct {
  double fs, gps_if, glo_if, mult, binw;
  int cbits, kbits, nch, iq, dev;
} g_cfg = {16.0e6, 2.42e6, 0.0, 5.0, 1000.0, 30, 29, 12, 1, 0};

static gnsscorr_track_ctx *g_ctx;
static gnsscorr_nco_cmd g_cmd[14];
static gnsscorr_track_result g_res[14];

static void die(const char *what, int rc)
{
  fprintf(stderr, "gnsscorr (OSG shim): %s failed (%d): %s\n", what, rc, gnsscorr_last_error());
  abort();
}

int gnsscorr_osg_configure(double samp_rate, double gps_if, double glonass_if,
                           double sys_clock_mult, int carrier_nco_bits, int code_nco_bits,
                           int n_channels, int use_iq, double freq_bin_width, int device)
{
  if (samp_rate <= 0 || sys_clock_mult <= 0 || carrier_nco_bits < 1 || carrier_nco_bits > 32 ||
      code_nco_bits < 1 || code_nco_bits > 32 || n_channels < 1 || n_channels > 14 || device < 0)
    return GNSSCORR_EINVAL;
  g_cfg.fs = samp_rate; g_cfg.gps_if = gps_if; g_cfg.glo_if = glonass_if;
  g_cfg.mult = sys_clock_mult; g_cfg.cbits = carrier_nco_bits; g_cfg.kbits = code_nco_bits;
  g_cfg.nch = n_channels; g_cfg.iq = use_iq ? 1 : 0; g_cfg.binw = freq_bin_width;
  g_cfg.dev = device;
  return GNSSCORR_OK;
}

void correlator_init(double tic_period)
{
  const char *e;
  if ((e = getenv("GNSSCORR_SAMP_RATE"))) g_cfg.fs = atof(e);
  if ((e = getenv("GNSSCORR_IF"))) g_cfg.gps_if = atof(e);
  if ((e = getenv("GNSSCORR_DEVICE"))) g_cfg.dev = atoi(e);

  /* correlator.c:110-121 */
  Carrier_DCO_Delta = g_cfg.mult * g_cfg.fs / pow(2.0, g_cfg.cbits);
  Code_DCO_Delta    = g_cfg.mult * g_cfg.fs / pow(2.0, g_cfg.kbits);
  gps_code_ref        = (long)(1023000 / Code_DCO_Delta);
  gps_carrier_ref     = (long)(g_cfg.gps_if / Carrier_DCO_Delta);
  glonass_code_ref    = (long)(511000 / Code_DCO_Delta);
  glonass_carrier_ref = (long)(g_cfg.glo_if / Carrier_DCO_Delta);
  d_freq              = (long)((int)g_cfg.binw / Carrier_DCO_Delta);

  /* gpchan is zeroed (correlator.c:128) but the ms/bit counters are file
   * statics the reference never resets: carry them over a re-init. */
  gnsscorr_chan_state keep[14];
  int have_keep = 0;
  if (g_ctx) {
    have_keep = gnsscorr_track_get_state(g_ctx, keep) == GNSSCORR_OK;
    gnsscorr_track_destroy(g_ctx);
    g_ctx = NULL;
  }
  gnsscorr_track_cfg tc;
  memset(&tc, 0, sizeof tc);
  tc.n_channels = g_cfg.nch;
  tc.iq = g_cfg.iq;
  tc.device = g_cfg.dev;
  tc.max_nsamp = 65536;
  tc.samp_rate = g_cfg.fs;
  tc.tic_period = tic_period;
  int rc = gnsscorr_track_create(&g_ctx, &tc);
  if (rc) die("gnsscorr_track_create", rc);
  if (have_keep) {
    gnsscorr_chan_state st[14];
    memset(st, 0, sizeof st);
    for (int ch = 0; ch < g_cfg.nch; ch++) {
      st[ch].ms_counter = keep[ch].ms_counter;
      st[ch].bit_counter = keep[ch].bit_counter;
      st[ch].msbit_reg = keep[ch].msbit_reg;
    }
    if ((rc = gnsscorr_track_set_state(g_ctx, st))) die("gnsscorr_track_set_state", rc);
  }
}

void Sim_GP2021_int(char *IF, long nsamp)
{
  if (!g_ctx) {
    fprintf(stderr, "gnsscorr (OSG shim): Sim_GP2021_int before correlator_init\n");
    abort();
  }
  const int nch = g_cfg.nch;
  for (int ch = 0; ch < nch; ch++) {
    const int reg = ch << 3;
    gnsscorr_nco_cmd *c = &g_cmd[ch];
    c->prn = REG_write[reg];
    if (c->prn > 32 || c->prn < 0) {
      fprintf(stderr, "gnsscorr (OSG shim): channel %d PRN %d outside 0..32 (the reference "
                      "would index past its 33-row code tables)\n", ch, c->prn);
      abort();
    }
    c->carrier_incr = ((uint32_t)REG_write[reg + 3] << 16) + (uint32_t)REG_write[reg + 4];
    c->code_incr    = ((uint32_t)REG_write[reg + 5] << 16) + (uint32_t)REG_write[reg + 6];
    c->slew         = (uint32_t)REG_write[(ch << 3) + 0x84] & 0xFFFFu;
    c->epoch_load   = REG_write[reg + 7] != -1 ? (REG_write[reg + 7] & 0xFFFF) : -1;
    c->stream       = 0;
  }
  int tic = 0;
  int rc = gnsscorr_track(g_ctx, (const int8_t *)IF, 0, 1, nsamp, g_cmd, g_res, NULL, &tic);
  if (rc) die("gnsscorr_track", rc);

  int status = 0;
  for (int ch = 0; ch < nch; ch++) {
    const int reg = ch << 3;
    const gnsscorr_track_result *r = &g_res[ch];
    if (g_cmd[ch].epoch_load != -1) REG_write[reg + 7] = -1;
    REG_read[reg + 7] = r->msbit_reg;
    if (r->n_dumps > 0) {
      for (int k = 0; k < 6; k++) REG_read[(ch << 3) + 0x84 + k] = r->dump[k];
      REG_write[(ch << 3) + 0x84] = 0;
      status |= 1 << ch;
    }
    if (r->tic)
      for (int k = 0; k < 6; k++) REG_read[reg + 1 + k] = r->tic_regs[k];
  }
  REG_read[0x82] = status;
  REG_read[0x83] = tic ? 0x2000 : 0x0;
}

int gnsscorr_osg_get_state(void *h_state_v)
{
  if (!g_ctx || !h_state_v) return GNSSCORR_EINVAL;
  return gnsscorr_track_get_state(g_ctx, (gnsscorr_chan_state *)h_state_v);
}
