/*
 * codes.c -- host-side code tables and the deterministic synthetic IF
 * generator (product code; no device work here).
 *
 *  gnsscorr_osg_table_image  E/P/L half-chip tables exactly as the OSGPS
 *                            correlator builds them (correlator.c:63-91),
 *                            laid out as one flat image so the reference's
 *                            row over-read (correlator.c:172-174, 247-251) is
 *                            reproduced (see DESIGN.md "over-read").
 *  gnsscorr_ca_code          SoftGNSS generateCAcode.sci:42-87 (ICD G2 delays)
 *  gnsscorr_st_code          SoftGNSS GLONASS generateSTcode.sci:35-42
 *  gnsscorr_sample_code      makeCaTable.sci:64-72 / makeStTable.sci:60-67
 *  gnsscorr_ifgen            int8 IQ at {-3,-1,1,3} (gps_source.cpp:692 levels)
 */
#include "gnsscorr_internal.h"
#include <pthread.h>
#include <stdlib.h>
#include <unistd.h>
#include <math.h>
#include <string.h>
#include <stdlib.h>

/* ---- OSG half-chip tables ----------------------------------------------- */
/* G2 register seeds per PRN (index 0 unused) -- the values OSGPS loads into
 * its 10-bit G2 shift register (correlator.c:67-71). */
static const uint16_t k_osg_g2_seed[33] = {
  0x000, 0x3f6, 0x3ec, 0x3d8, 0x3b0, 0x04b, 0x096, 0x2cb, 0x196, 0x32c, 0x3ba,
  0x374, 0x1d0, 0x3a0, 0x340, 0x280, 0x100, 0x113, 0x226, 0x04c, 0x098, 0x130,
  0x260, 0x267, 0x338, 0x270, 0x0e0, 0x1c0, 0x380, 0x22b, 0x056, 0x0ac, 0x158};

/* Chip sequence of one PRN with OSGPS conventions: chip 0 is forced to 1 and
 * chips 1..1022 are the first 1022 outputs of the G1^G2 generator seeded as
 * above (both registers shift right, feedback into bit 9). Values 0/1. */
static void osg_chips(int prn, uint8_t out[1023])
{
  unsigned g1 = 0x1FFu, g2 = k_osg_g2_seed[prn];
  out[0] = 1;
  for (int k = 1; k < 1023; k++) {
    out[k] = (uint8_t)((g1 ^ g2) & 1u);
    unsigned f1 = ((g1 >> 7) ^ g1) & 1u;                         /* taps 3,10 */
    unsigned f2 = ((g2 >> 8) ^ (g2 >> 7) ^ (g2 >> 4) ^ (g2 >> 2) ^ (g2 >> 1) ^ g2) & 1u;
    g1 = (g1 >> 1) | (f1 << 9);
    g2 = (g2 >> 1) | (f2 << 9);
  }
}

void gnsscorr_osg_table_image(int8_t *img)
{
  memset(img, 0, GNSSCORR_OSG_IMG_BYTES);
  for (int prn = 1; prn <= 32; prn++) {
    uint8_t c[1023];
    osg_chips(prn, c);
    int8_t *late = img + GNSSCORR_OSG_OFF_LATE + prn * GNSSCORR_OSG_ROW;
    int8_t *prompt = img + GNSSCORR_OSG_OFF_PROMPT + prn * GNSSCORR_OSG_ROW;
    int8_t *early = img + GNSSCORR_OSG_OFF_EARLY + prn * GNSSCORR_OSG_ROW;
    for (int h = 0; h < GNSSCORR_OSG_ROW; h++) {
      early[h]  = (int8_t)(c[h >> 1] ? 1 : -1);
      prompt[h] = (int8_t)(c[((h + 1) % GNSSCORR_OSG_ROW) >> 1] ? 1 : -1);
      late[h]   = (int8_t)(c[((h + 2) % GNSSCORR_OSG_ROW) >> 1] ? 1 : -1);
    }
  }
}

/* Packed table for the kernel: pk[b] = {late[b], prompt[b], early[b], 0} with
 * b = prn*2046 + index, read through the flat image so indices >= 2046 fall
 * into the following rows/tables exactly as the reference over-reads. */
void gnsscorr_osg_packed_table(uint32_t *pk)
{
  int8_t *img = (int8_t *)malloc(GNSSCORR_OSG_IMG_BYTES);
  gnsscorr_osg_table_image(img);
  for (int b = 0; b < GNSSCORR_OSG_PK_LEN; b++) {
    uint8_t l = (uint8_t)img[GNSSCORR_OSG_OFF_LATE + b];
    uint8_t p = (uint8_t)img[GNSSCORR_OSG_OFF_PROMPT + b];
    uint8_t e = (uint8_t)img[GNSSCORR_OSG_OFF_EARLY + b];
    pk[b] = (uint32_t)l | ((uint32_t)p << 8) | ((uint32_t)e << 16);
  }
  free(img);
}

/* ---- SoftGNSS codes ------------------------------------------------------ */
int gnsscorr_ca_code(int prn, int8_t *out)
{
  /* G2 delays per PRN, generateCAcode.sci:42-47 (first 32 entries used) */
  static const int g2s[32] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257, 258,
                              469, 470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516, 859, 860, 861, 862};
  if (prn < 1 || prn > 32 || !out) return GNSSCORR_EINVAL;
  int8_t g1[1023], g2[1023];
  int r1[10], r2[10];
  for (int i = 0; i < 10; i++) r1[i] = r2[i] = -1;
  for (int i = 0; i < 1023; i++) {                 /* +-1 product-form LFSRs */
    g1[i] = (int8_t)r1[9];
    int s1 = r1[2] * r1[9];
    g2[i] = (int8_t)r2[9];
    int s2 = r2[1] * r2[2] * r2[5] * r2[7] * r2[8] * r2[9];
    for (int k = 9; k > 0; k--) { r1[k] = r1[k - 1]; r2[k] = r2[k - 1]; }
    r1[0] = s1; r2[0] = s2;
  }
  int d = g2s[prn - 1];
  for (int i = 0; i < 1023; i++) {
    int j = (i - d + 1023) % 1023;                  /* g2 = [g2(end-d+1:end) g2(1:end-d)] */
    out[i] = (int8_t)(-(g1[i] * g2[j]));
  }
  return GNSSCORR_OK;
}

int gnsscorr_st_code(int8_t *out)
{
  if (!out) return GNSSCORR_EINVAL;
  int r[9];
  for (int i = 0; i < 9; i++) r[i] = -1;
  for (int i = 0; i < 511; i++) {
    int g3 = r[6];
    int s = r[4] * r[8];
    for (int k = 8; k > 0; k--) r[k] = r[k - 1];
    r[0] = s;
    out[i] = (int8_t)(-g3);
  }
  return GNSSCORR_OK;
}

int gnsscorr_sample_code(const int8_t *chips, int code_len, double code_rate, double fs,
                         int n, int8_t *out)
{
  if (!chips || !out || code_len <= 0 || n <= 0 || fs <= 0 || code_rate <= 0) return GNSSCORR_EINVAL;
  double ts = 1.0 / fs, tc = 1.0 / code_rate;
  for (int k = 1; k <= n; k++) {
    long idx = (long)ceil((ts * (double)k) / tc);   /* 1-based chip index */
    if (k == n) idx = code_len;                     /* codeValueIndex($) = codeLength */
    long j = ((idx - 1) % code_len + code_len) % code_len;
    out[k - 1] = chips[j];
  }
  return GNSSCORR_OK;
}

/* ---- synthetic IF ---------------------------------------------------------- */
typedef struct { uint64_t s; } lcg_t;
static inline uint64_t lcg_next(lcg_t *g)
{
  g->s = g->s * 6364136223846793005ULL + 1442695040888963407ULL;   /* MMIX LCG */
  return g->s;
}
static inline double lcg_unif(lcg_t *g) { return ((double)(lcg_next(g) >> 11) + 0.5) * (1.0 / 9007199254740992.0); }

static inline int8_t quant2(double x)
{
  /* 2-bit magnitude/sign quantiser, threshold at one noise sigma (== 1.0) */
  if (x >= 0) return (int8_t)(x < 1.0 ? 1 : 3);
  return (int8_t)(x > -1.0 ? -1 : -3);
}

/* g advanced by k steps of lcg_next (LCG jump-ahead by squaring) */
static uint64_t lcg_jump(uint64_t s, uint64_t k)
{
  uint64_t a = 6364136223846793005ULL, c = 1442695040888963407ULL, A = 1, C = 0;
  while (k) {
    if (k & 1) { A *= a; C = C * a + c; }
    c *= a + 1;
    a *= a;
    k >>= 1;
  }
  return s * A + C;
}

typedef struct {
  int8_t *out;
  int64_t nsamp;
  int iq;
  double fs;
  int n_sigs;
  const gnsscorr_sig *sigs;
  uint64_t seed;
  int8_t (*codes)[1023];
  int *clen;
  double *amp, *fcar, *crate, *bit_ms;
  uint32_t (*bits)[64];
  int64_t next;   /* next chunk (atomic) */
} ifgen_job;

#define IFGEN_CHUNK ((int64_t)1 << 18)

static void *ifgen_worker(void *arg)
{
  ifgen_job *j = (ifgen_job *)arg;
  const gnsscorr_sig *sigs = j->sigs;
  for (;;) {
    const int64_t n0 = __atomic_fetch_add(&j->next, IFGEN_CHUNK, __ATOMIC_RELAXED);
    if (n0 >= j->nsamp) break;
    const int64_t n1 = n0 + IFGEN_CHUNK < j->nsamp ? n0 + IFGEN_CHUNK : j->nsamp;
    lcg_t g = { lcg_jump(j->seed, 2 * (uint64_t)n0) };   /* two draws per sample */
    for (int64_t n = n0; n < n1; n++) {
      double t = (double)n / j->fs;
      double re = 0, im = 0;
      for (int s = 0; s < j->n_sigs; s++) {
        double chips = sigs[s].code_phase + t * j->crate[s];
        double per = floor(chips / j->clen[s]);
        long ci = (long)(chips - per * j->clen[s]);
        if (ci < 0) ci += j->clen[s];
        if (ci >= j->clen[s]) ci -= j->clen[s];
        double v = j->amp[s] * j->codes[s][ci];
        if (sigs[s].data_bits) {
          long bi = (long)floor(per * (1.0 / (j->bit_ms[s])));   /* one code period = 1 ms */
          bi = ((bi % 4096) + 4096) % 4096;
          if ((j->bits[s][(bi >> 5) & 63] >> (bi & 31)) & 1u) v = -v;
        }
        /* The reference front-end's complex IF is spectrum-inverted: the signal
         * sits at -f (acquisition.sci:107-111 and the GP2021 mixer,
         * correlator.c:213-215, both wipe off with exp(+i 2 pi f t)). */
        double ph = 2.0 * M_PI * j->fcar[s] * t + sigs[s].carr_phase;
        re += v * cos(ph);
        im -= v * sin(ph);
      }
      double u1 = lcg_unif(&g), u2 = lcg_unif(&g);
      double rad = sqrt(-2.0 * log(u1));
      double e1 = rad * cos(2.0 * M_PI * u2), e2 = rad * sin(2.0 * M_PI * u2);
      if (j->iq) {
        j->out[2 * n] = quant2(re + e1);
        j->out[2 * n + 1] = quant2(im + e2);
      } else {
        j->out[n] = quant2(re * 1.41421356237309505 + e1);
      }
    }
  }
  return NULL;
}

int gnsscorr_ifgen(int8_t *out, int64_t nsamp, int iq, double fs, double if_gps, double if_glo,
                   int n_sigs, const gnsscorr_sig *sigs, uint64_t seed)
{
  if (!out || nsamp <= 0 || fs <= 0 || n_sigs < 0 || (n_sigs > 0 && !sigs) || n_sigs > 64)
    return GNSSCORR_EINVAL;
  int8_t codes[64][1023];
  int    clen[64];
  double amp[64], fcar[64], crate[64], bit_ms[64];
  uint32_t bits[64][64];
  for (int s = 0; s < n_sigs; s++) {
    const gnsscorr_sig *g = &sigs[s];
    double f_rf;
    if (g->system == 0) {
      if (gnsscorr_ca_code(g->prn, codes[s]) != GNSSCORR_OK) return GNSSCORR_EINVAL;
      clen[s] = 1023; f_rf = 1575.42e6; crate[s] = 1.023e6; fcar[s] = if_gps + g->doppler;
      bit_ms[s] = 20.0;
    } else {
      gnsscorr_st_code(codes[s]);
      clen[s] = 511; f_rf = 1602.0e6 + g->fch * 0.5625e6; crate[s] = 0.511e6;
      fcar[s] = if_glo + g->fch * 0.5625e6 + g->doppler; bit_ms[s] = 10.0;
    }
    crate[s] *= (1.0 + g->doppler / f_rf);                   /* code Doppler */
    /* complex unit-variance-per-component noise: N0 = 2/fs; C = A^2 */
    amp[s] = sqrt(pow(10.0, g->cn0 / 10.0) * 2.0 / fs);
    lcg_t b = { seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(s + 1)) };
    for (int w = 0; w < 64; w++) bits[s][w] = g->data_bits ? (uint32_t)(lcg_next(&b) >> 32) : 0u;
  }
  ifgen_job job = {out, nsamp, iq, fs, n_sigs, sigs, seed ? seed : 0x5EED0000ULL, codes, clen,
                   amp, fcar, crate, bit_ms, bits, 0};
  /* chunks of samples over threads; each chunk starts its noise LCG by an
   * exact jump-ahead, so the output does not depend on the thread count */
  int nt = 1;
  const char *e = getenv("GNSSCORR_IFGEN_THREADS");
  if (e) nt = atoi(e);
  else {
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    nt = (int)(c > 16 ? 16 : c);
  }
  if (nt < 1) nt = 1;
  if (nsamp < (1 << 20)) nt = 1;
  pthread_t th[16];
  int started = 0;
  for (int i = 1; i < nt && i < 16; i++)
    if (pthread_create(&th[started], NULL, ifgen_worker, &job) == 0) started++;
  ifgen_worker(&job);
  for (int i = 0; i < started; i++) pthread_join(th[i], NULL);
  return GNSSCORR_OK;
}
