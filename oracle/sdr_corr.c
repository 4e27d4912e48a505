/*
 * oracle/sdr_corr.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the GPS-SDR tracking correlator
 * (REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER, "SDR/"):
 *
 *   sdrc_tables        Correlator::Correlator + SamplePRN, objects/correlator.cpp:63-98, 562-590
 *                      (carrier rows: sine_gen at -IF - 10 Hz * lcv; code rows: 101
 *                      fractional-chip bins per SV, fp32 phase accumulation)
 *   sdrc_accum         Correlator::Accum, correlator.cpp:425-448 (cmulsc shift 14 +
 *                      prn_accum_new, simd/x86.cpp:184-214, 359-386)
 *   sdrc_update        Correlator::UpdateState, correlator.cpp:369-422
 *   sdrc_dump          Correlator::DumpAccum, correlator.cpp:452-525 (fp64 rotation, floor)
 *   sdrc_correlate     Correlator::Correlate, correlator.cpp:160-237 (per 2048-sample packet)
 *   sdrc_init_chan     Correlator::InitCorrelator, correlator.cpp:610-676
 * The channel DLL/PLL (Channel::Accum) is host code outside the path: a
 * callback receives the rotated correlations and returns the NCO feedback.
 *
 * Parity: the primitives (sine_gen, code_gen, x86_cmulsc, x86_prn_accum_new) are
 * pinned against oracle/_ref/libsdr_ref.so (the reference sources built with
 * -DNO_SIMD); the Correlator class itself does not build standalone (threads,
 * pipes, usrp headers: SURVEY 8c), so its flow is restated line by line here.
 */
#include "sdr_corr.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

static const int k_delays[51] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257,
                                 258, 469, 470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516,
                                 859, 860, 861, 862, 145, 175, 52, 21, 237, 235, 886, 657, 634, 762,
                                 355, 1012, 176, 603, 130, 359, 595, 68, 386};

/* code_gen (accessories/misc.cpp:28-87): 0/1 chips of sv (0-based delay index) */
void sdrc_code_gen(int sv, uint8_t *chips)
{
  int g1[1023], g2[1023], r1[10], r2[10];
  for (int k = 0; k < 10; k++) r1[k] = r2[k] = 1;
  for (int k = 0; k < 1023; k++) {
    g1[k] = r1[0];
    g2[k] = r2[0];
    const int f1 = r1[7] ^ r1[0];
    const int f2 = (r2[8] + r2[7] + r2[4] + r2[2] + r2[1] + r2[0]) & 1;
    for (int j = 0; j < 9; j++) { r1[j] = r1[j + 1]; r2[j] = r2[j + 1]; }
    r1[9] = f1;
    r2[9] = f2;
  }
  unsigned d = 1023 - k_delays[sv];
  for (int k = 0; k < 1023; k++) {
    chips[k] = (uint8_t)(g1[k] ^ g2[d]);
    d = (d + 1) % 1023;
  }
}

void sdrc_tables(sdrc_cpx *carrier /* [SDRC_SBINS][SDRC_ROW] */,
                 int8_t *code /* [32][SDRC_CBINS][SDRC_ROW] */)
{
  if (carrier)
    for (int lcv = -SDRC_CARRIER_BINS; lcv <= SDRC_CARRIER_BINS; lcv++) {
      /* -IF_FREQUENCY-(float)lcv*CARRIER_SPACING is float arithmetic */
      const float f = (float)(-SDRC_IF) - (float)lcv * (float)SDRC_CARRIER_SPACING;
      sdro_sine_gen((sdro_cpx *)(carrier + (size_t)(lcv + SDRC_CARRIER_BINS) * SDRC_ROW), f,
                    SDRO_FS, SDRC_ROW);
    }
  if (code) {
    uint8_t chips[1023];
    for (int sv = 0; sv < 32; sv++) {
      sdrc_code_gen(sv, chips);
      for (int lcv = 0; lcv < SDRC_CBINS; lcv++) {
        int8_t *row = code + ((size_t)sv * SDRC_CBINS + lcv) * SDRC_ROW;
        float phase = (float)(-0.5 + (float)lcv / (float)SDRC_CODE_BINS);
        const float step = (float)(1.023e6 * 4.882812500000000e-7);
        for (int k = 0; k < SDRC_ROW; k++) {
          const int idx = (int)floorf(phase + 1023) % 1023;   /* C++ floor(float) */
          row[k] = chips[idx] ? 1 : -1;
          phase += step;
        }
      }
    }
  }
}

static inline int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }

void sdrc_accum(const sdrc_cpx *data, const sdrc_cpx *sine, const int8_t *e, const int8_t *p,
                const int8_t *l, int samps, int saturate, sdrc_corr *c)
{
  int32_t acc[6] = {0, 0, 0, 0, 0, 0};   /* E.i E.q P.i P.q L.i L.q (CPX_ACCUM int32) */
  for (int k = 0; k < samps; k++) {
    const int32_t ai = data[k].i, aq = data[k].q, bi = sine[k].i, bq = sine[k].q;
    int32_t ti = (ai * bi - aq * bq + 8192) >> 14, tq = (ai * bq + aq * bi + 8192) >> 14;
    const int32_t wi = saturate ? sat16(ti) : (int16_t)ti;
    const int32_t wq = saturate ? sat16(tq) : (int16_t)tq;
    acc[0] = (int32_t)((uint32_t)acc[0] + (uint32_t)(wi * e[k]));
    acc[1] = (int32_t)((uint32_t)acc[1] + (uint32_t)(wq * e[k]));
    acc[2] = (int32_t)((uint32_t)acc[2] + (uint32_t)(wi * p[k]));
    acc[3] = (int32_t)((uint32_t)acc[3] + (uint32_t)(wq * p[k]));
    acc[4] = (int32_t)((uint32_t)acc[4] + (uint32_t)(wi * l[k]));
    acc[5] = (int32_t)((uint32_t)acc[5] + (uint32_t)(wq * l[k]));
  }
  for (int j = 0; j < 3; j++) {
    c->I[j] = (int32_t)((uint32_t)c->I[j] + (uint32_t)acc[2 * j]);
    c->Q[j] = (int32_t)((uint32_t)c->Q[j] + (uint32_t)acc[2 * j + 1]);
  }
}

void sdrc_update(sdrc_state *s, int32_t samps)
{
  const double inv = 4.882812500000000e-7;   /* INVERSE_SAMPLE_FREQUENCY */
  s->code_phase += samps * s->code_nco * inv;
  s->carrier_phase += samps * s->carrier_nco * inv;
  s->code_phase_mod += samps * s->code_nco * inv;
  s->carrier_phase_mod += samps * s->carrier_nco * inv;
  int inc = s->code_phase_mod >= 2.0 * 1023.0 ? 2 : (s->code_phase_mod >= 1023.0 ? 1 : 0);
  if (inc) {
    s->_1ms_epoch += inc;
    if (s->_1ms_epoch >= 20) {
      s->_1ms_epoch %= 20;
      s->_20ms_epoch++;
      if (s->_20ms_epoch >= 300) {
        s->_20ms_epoch = 0;
        s->_z_count += 6;
        if (s->_z_count > 604800.0) s->_z_count = 0;
      }
    }
  }
  s->carrier_phase_mod = fmod(s->carrier_phase_mod, 1.0);
  s->code_phase_mod = fmod(s->code_phase_mod, 1023);
  s->rollover -= (uint32_t)samps;
  s->soff += samps;
  for (int j = 0; j < 3; j++) s->coff[j] += samps;
  s->scount += (uint32_t)samps;
}

static uint32_t code_bin(double phase)
{
  int32_t b = (int32_t)floor(phase * SDRC_CODE_BINS + 0.5) + SDRC_CODE_BINS / 2;
  if (b < 0) b = 0;
  if (b > 2 * SDRC_CODE_BINS) b = 2 * SDRC_CODE_BINS;
  return (uint32_t)b;
}

static uint32_t carrier_bin(double nco)
{
  int32_t b = (int32_t)floor((nco - SDRC_IF) / SDRC_CARRIER_SPACING + 0.5) + SDRC_CARRIER_BINS;
  if (b < 0) b = 0;
  if (b > 2 * SDRC_CARRIER_BINS) b = 2 * SDRC_CARRIER_BINS;
  return (uint32_t)b;
}

void sdrc_rotate(sdrc_state *s, sdrc_corr *c)
{
  /* f1 is computed in uint32 in the reference ((sbin - CARRIER_BINS) with sbin
   * uint32): bins below the centre wrap to ~4.29e9 Hz -- reproduced. */
  const double f1 = (double)((s->sbin - (uint32_t)SDRC_CARRIER_BINS) * (uint32_t)SDRC_CARRIER_SPACING +
                             (uint32_t)SDRC_IF);
  const double f2 = s->carrier_nco;
  const double fix = 3.141592653589793 * (f2 - f1) * (double)s->scount * 4.882812500000000e-7;
  double ang = s->carrier_phase_prev * 6.283185307179586 + fix;
  ang = -ang;
  const double ca = cos(ang), sa = sin(ang);
  s->carrier_phase_prev = s->carrier_phase_mod;
  for (int j = 0; j < 3; j++) {
    const double tI = c->I[j], tQ = c->Q[j];
    c->I[j] = (int32_t)floor(ca * tI - sa * tQ);
    c->Q[j] = (int32_t)floor(sa * tI + ca * tQ);
  }
}

void sdrc_feedback_apply(sdrc_state *s, const sdrc_feedback *f)
{
  s->carrier_nco = f->carrier_nco;
  s->code_nco = f->code_nco;
  s->navigate = f->navigate;
  if (f->reset_1ms) s->_1ms_epoch = 0;
  if (f->reset_20ms) s->_20ms_epoch = 60;
  if (f->set_z_count) s->_z_count = f->z_count;
  if (f->kill) memset(s, 0, sizeof *s);
}

void sdrc_rebin(sdrc_state *s)
{
  /* (int32) of an infinite rollover (code_nco 0 after a kill) is INT_MIN on x86 */
  const double r = ceil(((double)1023 - s->code_phase_mod) * 2048000.0 / s->code_nco);
  s->rollover = isfinite(r) ? (uint32_t)(int32_t)r : 0x80000000u;
  s->cbin[0] = code_bin(s->code_phase_mod + 0.5);
  s->cbin[1] = code_bin(s->code_phase_mod + 0.0);
  s->cbin[2] = code_bin(s->code_phase_mod - 0.5);
  s->coff[0] = s->coff[1] = s->coff[2] = 0;
  s->sbin = carrier_bin(s->carrier_nco);
  s->soff = 0;
  s->scount = 0;
}

static void dump(sdrc_state *s, sdrc_corr *c, int ch, sdrc_cb cb, void *user)
{
  sdrc_rotate(s, c);
  sdrc_feedback f;
  memset(&f, 0, sizeof f);
  cb(user, ch, s, c, &f);            /* Channel::Accum (host DLL/PLL) */
  sdrc_feedback_apply(s, &f);
  s->count++;
  memset(c, 0, sizeof *c);
  sdrc_rebin(s);   /* also after a kill: bins from the zeroed state, as the reference */
}

static void accum_seg(const sdrc_tables_t *t, const sdrc_cpx *data, sdrc_state *s, int samps,
                      int saturate, sdrc_corr *c)
{
  if (samps <= 0) return;
  const sdrc_cpx *sine = t->carrier + (size_t)s->sbin * SDRC_ROW + s->soff;
  const int8_t *rows = t->code + (size_t)s->sv * SDRC_CBINS * SDRC_ROW;
  sdrc_accum(data, sine, rows + (size_t)s->cbin[0] * SDRC_ROW + s->coff[0],
             rows + (size_t)s->cbin[1] * SDRC_ROW + s->coff[1],
             rows + (size_t)s->cbin[2] * SDRC_ROW + s->coff[2], samps, saturate, c);
}

void sdrc_correlate(const sdrc_tables_t *t, const sdrc_cpx *packet, int n_ch, sdrc_state *st,
                    sdrc_corr *corr, int saturate, sdrc_cb cb, void *user)
{
  for (int ch = 0; ch < n_ch; ch++) {
    sdrc_state *s = &st[ch];
    sdrc_corr *c = &corr[ch];
    if (!s->active) continue;
    const sdrc_cpx *d = packet;
    int32_t left = SDRC_N;
    if (s->rollover <= (uint32_t)SDRC_N) {
      const int32_t r1 = (int32_t)s->rollover;
      accum_seg(t, d, s, r1, saturate, c);
      left = SDRC_N - r1;
      d += r1;
      sdrc_update(s, r1);
      dump(s, c, ch, cb, user);
      if (!s->active) continue;
      if (s->rollover <= (uint32_t)left) {
        const int32_t r2 = (int32_t)s->rollover;
        accum_seg(t, d, s, r2, saturate, c);
        left -= r2;
        d += r2;
        sdrc_update(s, r2);
        dump(s, c, ch, cb, user);
        if (!s->active) continue;
        accum_seg(t, d, s, left, saturate, c);
        sdrc_update(s, left);
      } else {
        accum_seg(t, d, s, left, saturate, c);
        sdrc_update(s, left);
      }
    } else {
      accum_seg(t, d, s, SDRC_N, saturate, c);
      sdrc_update(s, SDRC_N);
    }
  }
}

void sdrc_init_chan(sdrc_state *s, int sv, int acq_code_phase, int acq_doppler,
                    double packets_since_acq)
{
  memset(s, 0, sizeof *s);
  double dt = packets_since_acq;
  dt *= (double).001;
  dt *= (double)acq_doppler * (double)1.023e6 / (double)1.57542e9;
  double cp = (double)acq_code_phase * 1023.0 / 2048.0;
  cp += (double)1023 - dt + 2.5;
  cp = fmod(cp, (double)1023);
  s->sv = (uint32_t)sv;
  s->active = 1;
  s->code_phase = s->code_phase_mod = cp;
  s->code_nco = 1.023e6 + acq_doppler * 1.023e6 / 1.57542e9;
  s->carrier_nco = SDRC_IF + acq_doppler;
  s->rollover = (uint32_t)(int32_t)ceil(((double)1023 - cp) * 2048000.0 / s->code_nco);
  s->cbin[0] = code_bin(cp + 0.5);
  s->cbin[1] = code_bin(cp + 0.0);
  s->cbin[2] = code_bin(cp - 0.5);
  for (int j = 0; j < 3; j++) s->coff[j] = acq_code_phase;   /* pcode[k] += inc */
  s->sbin = carrier_bin(s->carrier_nco);
  s->soff = 0;
}

/* A deterministic stand-in for Channel::Accum used by the parity tests: a
 * first-order carrier/code discriminator loop on the prompt arm, plus (user =
 * int[2] {kill_after, kill_sv}) a kill of the channel tracking sv kill_sv
 * after kill_after dumps when kill_after > 0. */
void sdrc_test_loop(void *user, int ch, const sdrc_state *s, const sdrc_corr *c,
                    sdrc_feedback *f)
{
  const int kill_after = user ? ((const int *)user)[0] : 0;
  const int kill_sv = user ? ((const int *)user)[1] : -1;
  const double ip = c->I[1], qp = c->Q[1];
  const double e = sqrt((double)c->I[0] * c->I[0] + (double)c->Q[0] * c->Q[0]);
  const double l = sqrt((double)c->I[2] * c->I[2] + (double)c->Q[2] * c->Q[2]);
  const double perr = ip != 0.0 ? atan(qp / ip) : 0.0;
  const double derr = (e + l) > 0 ? (e - l) / (e + l) : 0.0;
  f->carrier_nco = s->carrier_nco + 2.0 * perr;
  f->code_nco = s->code_nco + 0.5 * derr;
  f->navigate = 1;
  f->reset_1ms = (s->count % 97) == 5;
  f->kill = kill_after > 0 && (int)s->sv == kill_sv && (int)s->count + 1 >= kill_after;
  (void)ch;
}
