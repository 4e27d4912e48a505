/*
 * oracle/osg_corr.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * A deliberately literal, sample-by-sample restatement of the OSGPS software
 * GP2021 correlator:
 *   generate_gps_prn_codes  osgnss_next_step/src/correlator/correlator.c:63-91
 *   correlator_init         correlator.c:107-132
 *   Sim_GP2021_int          correlator.c:148-316
 *   ch_* accessors          osgnss_next_step/src/gp2021/gp2021.c:11-130
 * Pinned bit-exact against the reference compiled from its own sources
 * (oracle/_ref/libosg_ref.so) by tests/test_oracle_osg.py.
 *
 * Over-read quirk (correlator.c:172-174, 247-251): when the code rollover that
 * triggers a dump happens, the E/P/L bits are re-loaded from index
 * half_chip >= 2046 of the PRN's row, i.e. from the next row of the same
 * table (row-major), before half_chip is reset to 0 without a reload.  To be
 * bit-exact this restatement keeps the three tables in ONE flat image laid
 * out exactly as gcc places the reference's three statics (observed with
 * `nm -n` on oracle/_ref/libosg_ref.so):  late[33][2046] | 2 pad bytes |
 * prompt[33][2046] | 2 pad | early[33][2046] | zeros.  Row 0 of every table is
 * never generated (prn loop starts at 1) and stays zero.
 */
#include "osg_corr.h"
#include <string.h>
#include <stdlib.h>
#include <math.h>
#include <pthread.h>

#define ROW        2046
#define NROWS      33
#define TAB        (ROW * NROWS)           /* 67518 bytes per table */
#define OFF_LATE   0
#define OFF_PROMPT (TAB + 2)                /* 67520 */
#define OFF_EARLY  (2 * (TAB + 2))          /* 135040 */
#define IMG_BYTES  (OFF_EARLY + 32 * ROW + 65536 + 2048 + 256)

static int8_t g_img[IMG_BYTES];
static int    g_img_ready;

static void build_tables(void)
{
  /* G2 initial states, correlator.c:67-71 (standard GPS ICD G2 phase selects
   * expressed as register seeds). */
  static const int G2_i[33] = {
    0x000, 0x3f6, 0x3ec, 0x3d8, 0x3b0, 0x04b, 0x096, 0x2cb, 0x196,
    0x32c, 0x3ba, 0x374, 0x1d0, 0x3a0, 0x340, 0x280, 0x100,
    0x113, 0x226, 0x04c, 0x098, 0x130, 0x260, 0x267, 0x338,
    0x270, 0x0e0, 0x1c0, 0x380, 0x22b, 0x056, 0x0ac, 0x158};
  memset(g_img, 0, sizeof g_img);
  for (int prn = 1; prn < 33; prn++) {
    int8_t c[1023];
    int g1 = 0x1FF, g2 = G2_i[prn];
    c[0] = 1;                                   /* forced, correlator.c:75 */
    for (int k = 1; k < 1023; k++) {
      c[k] = (int8_t)((g1 ^ g2) & 1);
      int fb1 = ((g1 << 2) ^ (g1 << 9)) & 0x200;
      g1 = (g1 >> 1) | fb1;
      int fb2 = ((g2 << 1) ^ (g2 << 2) ^ (g2 << 5) ^ (g2 << 7) ^ (g2 << 8) ^ (g2 << 9)) & 0x200;
      g2 = (g2 >> 1) | fb2;
    }
    for (int h = 0; h < ROW; h++) {
      g_img[OFF_EARLY  + prn * ROW + h] = (int8_t)(2 * c[((h + 0) % ROW) >> 1] - 1);
      g_img[OFF_PROMPT + prn * ROW + h] = (int8_t)(2 * c[((h + 1) % ROW) >> 1] - 1);
      g_img[OFF_LATE   + prn * ROW + h] = (int8_t)(2 * c[((h + 2) % ROW) >> 1] - 1);
    }
  }
  g_img_ready = 1;
}

int  osgo_table_bytes(void) { return IMG_BYTES; }
void osgo_table_image(int8_t *out) { if (!g_img_ready) build_tables(); memcpy(out, g_img, IMG_BYTES); }
int  osgo_sizeof(void) { return (int)sizeof(osgo_t); }

void osgo_init(osgo_t *o, int n_channels, int use_iq, double samp_rate, double tic_period)
{
  if (!g_img_ready) build_tables();
  memset(o, 0, sizeof *o);
  o->n_channels = n_channels;
  o->use_iq = use_iq;
  /* correlator.c:124-125: tic_ref = SAMP_RATE * tic_period (long) */
  o->tic_ref = (int64_t)(samp_rate * tic_period);
  o->tic = o->tic_ref;
}

/* ---- gp2021.c register accessors (host side of the boundary) ---------- */
static void outpwd(osgo_t *o, int add, int data) { o->reg_write[add & 0xFF] = (uint16_t)data; }
void osgo_ch_cntl(osgo_t *o, int ch, int prn) { outpwd(o, ch << 3, prn); }
void osgo_ch_code_slew(osgo_t *o, int ch, int slew) { outpwd(o, (ch << 3) + 0x84, slew); }
void osgo_ch_epoch_load(osgo_t *o, int ch, unsigned data) { outpwd(o, (ch << 3) + 7, (int)data); }
void osgo_ch_carrier(osgo_t *o, int ch, long freq)
{
  /* gp2021.c:81-100: (freq << (32-30)) * 5.0, split hi/lo 16 */
  long f = (long)((double)(freq << 2) * 5.0);
  outpwd(o, (ch << 3) + 3, (int)(f >> 16));
  outpwd(o, (ch << 3) + 4, (int)(f & 0xffff));
}
void osgo_ch_code(osgo_t *o, int ch, long freq)
{
  long f = (long)((double)(freq << 3) * 5.0);  /* gp2021.c:102-120 */
  outpwd(o, (ch << 3) + 5, (int)(f >> 16));
  outpwd(o, (ch << 3) + 6, (int)(f & 0xffff));
}
int osgo_reg_read(const osgo_t *o, int addr) { return (short)o->reg_read[addr & 0xFF]; }

/* Optional log of every dump (test-only: the reference latches only the last
 * dump of a call in REG_read); entries {ch, IL, QL, IP, QP, IE, QE}. */
static int32_t *g_dlog;
static int g_dcap, g_dn;
void osgo_dump_log(int32_t *buf, int cap) { g_dlog = buf; g_dcap = cap; g_dn = 0; }
int  osgo_dump_count(void) { return g_dn; }

/* ---- Sim_GP2021_int restated (correlator.c:148-316) --------------------- */
void osgo_sim(osgo_t *o, const int8_t *IF, long nsamp)
{
  static const int i_lo[8] = {-1, 1, 2, 2, 1, -1, -2, -2};   /* :203 */
  static const int q_lo[8] = { 2, 2, 1, -1, -2, -2, -1, 1};  /* :204 */
  long tic_count;
  if (o->tic < nsamp) { tic_count = (long)o->tic; o->tic += o->tic_ref - nsamp; }
  else                { o->tic -= nsamp; tic_count = -1; }

  int status = 0;
  for (int ch = 0; ch < o->n_channels; ch++) {
    int reg = ch << 3;
    int slew_dump = o->reg_write[(ch << 3) + 0x84] + 2046;
    if (o->reg_write[reg + 7] != -1) {                       /* epoch load :177-182 */
      o->reg_read[reg + 7] = o->reg_write[reg + 7];
      o->ms_counter[ch]  = o->reg_write[reg + 7] & 0xff;
      o->bit_counter[ch] = o->reg_write[reg + 7] >> 8;
      o->reg_write[reg + 7] = -1;
    }
    int prn = o->reg_write[reg];
    if (prn <= 0) continue;
    uint32_t cinc = ((uint32_t)o->reg_write[reg + 3] << 16) + (uint32_t)o->reg_write[reg + 4];
    uint32_t kinc = ((uint32_t)o->reg_write[reg + 5] << 16) + (uint32_t)o->reg_write[reg + 6];
    const int8_t *E = g_img + OFF_EARLY + prn * ROW;
    const int8_t *P = g_img + OFF_PROMPT + prn * ROW;
    const int8_t *L = g_img + OFF_LATE + prn * ROW;
    const int8_t *ifp = IF;
    int pb = P[o->half_chip[ch]], lb = L[o->half_chip[ch]], eb = E[o->half_chip[ch]];
    int32_t *a = o->acc[ch];
    for (long i = 0; i < nsamp; i++) {
      int idx = (int)(o->carrier_phase[ch] >> 29);
      int ival, qval;
      if (o->use_iq) {
        int ti = *ifp++, tq = *ifp++;
        qval = q_lo[idx] * ti - i_lo[idx] * tq;
        ival = i_lo[idx] * ti + q_lo[idx] * tq;
      } else {
        int t = *ifp++;
        ival = t * i_lo[idx];
        qval = t * q_lo[idx];
      }
      /* int32 wrap-around accumulation (unsigned arithmetic = defined wrap) */
      a[1] = (int32_t)((uint32_t)a[1] + (uint32_t)(lb * qval));
      a[3] = (int32_t)((uint32_t)a[3] + (uint32_t)(pb * qval));
      a[5] = (int32_t)((uint32_t)a[5] + (uint32_t)(eb * qval));
      a[0] = (int32_t)((uint32_t)a[0] + (uint32_t)(lb * ival));
      a[2] = (int32_t)((uint32_t)a[2] + (uint32_t)(pb * ival));
      a[4] = (int32_t)((uint32_t)a[4] + (uint32_t)(eb * ival));
      uint32_t cr = o->carrier_phase[ch];
      o->carrier_phase[ch] += cinc;
      if (o->carrier_phase[ch] < cr) o->carrier_cycle[ch]++;
      uint32_t kr = o->code_phase[ch];
      o->code_phase[ch] += (kinc << 1);
      if (o->code_phase[ch] < kr) {
        o->half_chip[ch]++;
        uint16_t h = o->half_chip[ch];
        pb = P[h]; lb = L[h]; eb = E[h];
        if (h >= slew_dump) {
          int r = (ch << 3) + 0x84;
          for (int k = 0; k < 6; k++) o->reg_read[r + k] = a[k];
          if (g_dlog && g_dn < g_dcap) {
            g_dlog[7 * g_dn] = ch;
            for (int k = 0; k < 6; k++) g_dlog[7 * g_dn + 1 + k] = a[k];
            g_dn++;
          }
          o->reg_write[r] = 0;
          for (int k = 0; k < 6; k++) a[k] = 0;
          o->half_chip[ch] = 0;
          status |= 1 << ch;
          o->ms_counter[ch]++;
          if (o->ms_counter[ch] == 20) o->bit_counter[ch] = (o->bit_counter[ch] + 1) % 50;
          o->ms_counter[ch] %= 20;
          o->reg_read[ch * 8 + 7] = o->ms_counter[ch] + (o->bit_counter[ch] << 8);
        }
      }
      if (i == tic_count) {
        int r = ch << 3;
        o->reg_read[r + 4] = o->reg_read[r + 7];
        o->reg_read[r + 3] = (int32_t)(o->carrier_phase[ch] >> 22);
        o->reg_read[r + 1] = o->half_chip[ch];
        o->reg_read[r + 5] = (int32_t)(o->code_phase[ch] >> 22);
        o->reg_read[r + 2] = (int32_t)(o->carrier_cycle[ch] & 0xffff);
        o->reg_read[r + 6] = (int32_t)(o->carrier_cycle[ch] >> 16);
        o->carrier_cycle[ch] = 0;
      }
    }
  }
  o->reg_read[0x82] = status;
  o->reg_read[0x83] = (tic_count > -1) ? 0x2000 : 0;
}

/* ---- threaded CPU baseline ------------------------------------------------ */
typedef struct {
  int first, last, n_channels, n_calls, if_calls; long nsamp; const int8_t *IF;
  long cf, kf; double work;
} job_t;

static void *bench_worker(void *arg)
{
  job_t *j = (job_t *)arg;
  osgo_t *o = (osgo_t *)malloc(sizeof(osgo_t));
  for (int inst = j->first; inst < j->last; inst++) {
    osgo_init(o, j->n_channels, 1, 16.368e6, 0.0);
    for (int ch = 0; ch < j->n_channels; ch++) {
      osgo_ch_cntl(o, ch, 1 + (inst * j->n_channels + ch) % 32);
      osgo_ch_carrier(o, ch, j->cf + 13 * ch);
      osgo_ch_code(o, ch, j->kf);
    }
    const int8_t *base = j->IF + (size_t)inst * (size_t)j->if_calls * (size_t)j->nsamp * 2;
    for (int c = 0; c < j->n_calls; c++) {
      osgo_sim(o, base + (size_t)(c % j->if_calls) * (size_t)j->nsamp * 2, j->nsamp);
      j->work += (double)j->n_channels * (double)j->nsamp;
    }
  }
  free(o);
  return NULL;
}

double osgo_bench(int n_inst, int n_channels, const int8_t *IF, long nsamp, int n_calls,
                  int if_calls, long carrier_freq, long code_freq, int threads)
{
  if (!g_img_ready) build_tables();
  if (threads < 1) threads = 1;
  if (threads > n_inst) threads = n_inst;
  pthread_t th[256]; job_t jobs[256];
  if (threads > 256) threads = 256;
  for (int t = 0; t < threads; t++) {
    jobs[t].first = (int)((long)n_inst * t / threads);
    jobs[t].last  = (int)((long)n_inst * (t + 1) / threads);
    jobs[t].n_channels = n_channels; jobs[t].n_calls = n_calls; jobs[t].nsamp = nsamp;
    jobs[t].if_calls = if_calls;
    jobs[t].IF = IF; jobs[t].cf = carrier_freq; jobs[t].kf = code_freq; jobs[t].work = 0;
    pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
  }
  double w = 0;
  for (int t = 0; t < threads; t++) { pthread_join(th[t], NULL); w += jobs[t].work; }
  return w;
}
