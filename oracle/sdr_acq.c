/*
 * oracle/sdr_acq.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the GPS-SDR strong (1 ms) acquisition, the
 * integer-FFT acquisition of the real-time receiver
 * (REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER, "SDR/"):
 *
 *   sdro_sine_gen      SDR/accessories/misc.cpp:95-115 (fp32 phase accumulator)
 *   sdro_fft           SDR/objects/fft.cpp:114-245 (twiddles, bit reverse, DIT ranks),
 *                      scalar butterflies fft.cpp:403-441 (the -DNO_SIMD path)
 *   sdro_cmulsc        SDR/simd/x86.cpp:184-214 (wrap) / sse.cpp:646-729 (packssdw saturate)
 *   sdro_cmag/max      SDR/simd/x86.cpp:250-288
 *   sdro_prep_if       Acquisition::doPrepIF, SDR/objects/acquisition.cpp:191-236 (1 ms)
 *   sdro_acq_strong    Acquisition::doAcqStrong, acquisition.cpp:244-301
 *   sdro_prn_codes     SDR/accessories/gen_fft_codes.m + prn_gen.m (the PRN_Codes table)
 *   sdro_wipeoff_gen   SDR/accessories/misc.cpp:148-168 (fp64 phase, MIX rows)
 *   sdro_cacc          SDR/simd/x86.cpp:220-249 (= sse_cacc, sse.cpp:732-800)
 *   sdro_prep_rows     Acquisition::doPrepIF for 1 / 10 / 310 ms (acquisition.cpp:191-236)
 *                      into the persistent baseband_rows store (1240 rows)
 *   sdro_acq_medium    Acquisition::doAcqMedium, acquisition.cpp:309-425
 *   sdro_acq_weak      Acquisition::doAcqWeak, acquisition.cpp:433-570
 *
 * Parity pinned: tests/test_oracle_sdr.py checks every function against the
 * reference primitives compiled from their own sources with -DNO_SIMD
 * (oracle/_ref/libsdr_ref.so, see oracle/Makefile) and against the committed
 * fixtures in tests/golden/ (PRN_Codes from prn_codes.h, acquisition results
 * of the reference build).  Used by tests/ and bench.py's cpu_baseline only.
 */
#include "sdr_acq.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define SDRO_TWO_PI 6.283185307179586 /* defines.h:104 */

void sdro_sine_gen(sdro_cpx *dst, double f, double fs, int n)
{
  float phase = 0.0f;
  const float step = (float)SDRO_TWO_PI * f / fs;   /* float * double / double -> float */
  for (int k = 0; k < n; k++) {
    /* misc.cpp is C++: cos(float) is the float overload (cosf) */
    dst[k].i = (int16_t)floor(16383.0 * (double)cosf(phase));
    dst[k].q = (int16_t)floor(16383.0 * (double)sinf(phase));
    phase += step;
  }
}

void sdro_twiddles(int n, sdro_mix *w, sdro_mix *iw)
{
  const double pi = 3.14159265358979323846264338327;
  for (int k = 0; k < n / 2; k++) {
    const double ph = (-2 * pi * k) / n;
    const double c = floor(16384 * cos(ph)), s = floor(16384 * sin(ph));
    w[k].i = (int16_t)c;  w[k].q = (int16_t)s;  w[k].nq = (int16_t)(-s); w[k].ni = (int16_t)c;
    iw[k].i = (int16_t)c; iw[k].q = (int16_t)(-s); iw[k].nq = (int16_t)s; iw[k].ni = (int16_t)c;
  }
}

static int ilog2(int n) { int m = 0; while (n > 1) { m++; n >>= 1; } return m; }

static int bitrev(int v, int m)
{
  int r = 0;
  for (int b = 0; b < m; b++) r = (r << 1) | ((v >> b) & 1);
  return r;
}

/* one radix-2 DIT butterfly, optional pre-scaling by 1/2 (fft.cpp:403-441) */
static void bfly(sdro_cpx *a, sdro_cpx *b, const sdro_mix *w, int scale)
{
  if (scale) {
    a->i >>= 1; a->q >>= 1; b->i >>= 1; b->q >>= 1;
  }
  int32_t bi = b->i * w->i - b->q * w->q;
  int32_t bq = b->i * w->q + b->q * w->i;
  bi = (bi + 8192) >> 14;
  bq = (bq + 8192) >> 14;
  b->i = (int16_t)(a->i - (int16_t)bi);
  b->q = (int16_t)(a->q - (int16_t)bq);
  a->i = (int16_t)(a->i + (int16_t)bi);
  a->q = (int16_t)(a->q + (int16_t)bq);
}

void sdro_fft(sdro_cpx *x, int n, const sdro_mix *w, const int32_t *rank_scale)
{
  const int m = ilog2(n);
  sdro_cpx *tmp = (sdro_cpx *)malloc(sizeof(sdro_cpx) * n);
  memcpy(tmp, x, sizeof(sdro_cpx) * n);
  for (int k = 0; k < n; k++) x[k] = tmp[bitrev(k, m)];      /* doShuffle */
  free(tmp);
  int bsize = 1, nblocks = n >> 1;
  for (int r = 0; r < m; r++) {
    for (int blk = 0; blk < nblocks; blk++)
      for (int j = 0; j < bsize; j++)
        bfly(&x[blk * 2 * bsize + j], &x[blk * 2 * bsize + j + bsize], &w[j * nblocks],
             rank_scale[r]);
    bsize <<= 1;
    nblocks >>= 1;
  }
}

static inline int16_t sat16(int32_t v) { return (int16_t)(v > 32767 ? 32767 : v < -32768 ? -32768 : v); }

void sdro_cmulsc(const sdro_cpx *a, const sdro_cpx *b, sdro_cpx *c, int n, int shift, int saturate)
{
  const int32_t round = 1 << (shift - 1);
  for (int k = 0; k < n; k++) {
    const int32_t ai = a[k].i, aq = a[k].q, bi = b[k].i, bq = b[k].q;
    int32_t ti = ai * bi - aq * bq, tq = ai * bq + aq * bi;
    ti = (ti + round) >> shift;
    tq = (tq + round) >> shift;
    c[k].i = saturate ? sat16(ti) : (int16_t)ti;
    c[k].q = saturate ? sat16(tq) : (int16_t)tq;
  }
}

void sdro_cmag_max(const sdro_cpx *a, int n, int32_t *index, int32_t *mag)
{
  int32_t best = 0, idx = 0;
  for (int k = 0; k < n; k++) {
    const int32_t p = (int32_t)((uint32_t)(a[k].i * a[k].i) + (uint32_t)(a[k].q * a[k].q));
    if (p > best) { best = p; idx = k; }
  }
  *index = idx;
  *mag = best;
}

void sdro_prep_if(const sdro_cpx *buff, double fif, int saturate, sdro_cpx rows[4][SDRO_N])
{
  sdro_cpx wipe[4][SDRO_N];
  sdro_mix w[SDRO_N / 2], iw[SDRO_N / 2];
  static const int32_t r1[16] = {0};
  for (int j = 0; j < 4; j++) sdro_sine_gen(wipe[j], -fif - 250.0 * j, SDRO_FS, SDRO_N);
  /* rows 1..3 from the raw buffer, then row 0 mixed in place (acquisition.cpp:216-222) */
  for (int j = 1; j < 4; j++) sdro_cmulsc(buff, wipe[j], rows[j], SDRO_N, 14, saturate);
  sdro_cmulsc(buff, wipe[0], rows[0], SDRO_N, 14, saturate);
  sdro_twiddles(SDRO_N, w, iw);
  for (int j = 0; j < 4; j++) sdro_fft(rows[j], SDRO_N, w, r1);
}

sdro_result sdro_acq_strong(sdro_cpx rows[4][SDRO_N], const sdro_cpx *code, int sv, int doppmin,
                            int doppmax, int saturate)
{
  static const int32_t r2[16] = {0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 1};
  sdro_mix w[SDRO_N / 2], iw[SDRO_N / 2];
  sdro_twiddles(SDRO_N, w, iw);
  sdro_result r;
  memset(&r, 0, sizeof r);
  r.sv = sv;
  int32_t mag = 0;
  sdro_cpx sh[SDRO_N], buf[SDRO_N];
  for (int lcv = doppmin / 1000; lcv < doppmax / 1000; lcv++)
    for (int lcv2 = 0; lcv2 < 4; lcv2++) {
      /* baseband_rows[lcv2][100 + lcv]: the row read circularly from offset lcv */
      for (int k = 0; k < SDRO_N; k++) sh[k] = rows[lcv2][(k + lcv + SDRO_N) & (SDRO_N - 1)];
      sdro_cmulsc(sh, code, buf, SDRO_N, 10, saturate);
      sdro_fft(buf, SDRO_N, iw, r2);
      int32_t idx, m;
      sdro_cmag_max(buf, SDRO_N, &idx, &m);
      if (m > mag) {
        mag = m;
        r.code_phase = SDRO_N - idx;
        r.doppler = lcv * 1000 + lcv2 * 250;
        r.magnitude = (uint32_t)m;
        r.row = (lcv - doppmin / 1000) * 4 + lcv2;
      }
    }
  r.success = r.magnitude > 0;   /* THRESH_STRONG = 0 (config.h:72) */
  return r;
}

/* ---- medium / weak acquisition ------------------------------------------ */
void sdro_wipeoff_gen(sdro_mix *dst, double f, double fs, int n)
{
  double phase = 0.0;
  const double step = SDRO_TWO_PI * f / fs;
  for (int k = 0; k < n; k++) {
    const int16_t c = (int16_t)floor(16383.0 * cos(phase));
    const int16_t s = (int16_t)floor(16383.0 * sin(phase));
    dst[k].i = dst[k].ni = c;
    dst[k].q = s;
    dst[k].nq = (int16_t)(-s);
    phase += step;
  }
}

void sdro_cacc(const sdro_cpx *a, const sdro_mix *b, int n, int32_t *iacc, int32_t *qacc)
{
  uint32_t ia = 0, qa = 0;                     /* int32 wrap, as paddd */
  for (int k = 0; k < n; k++) {
    ia += (uint32_t)(a[k].i * b[k].i + a[k].q * b[k].nq);
    qa += (uint32_t)(a[k].i * b[k].q + a[k].q * b[k].ni);
  }
  *iacc = (int32_t)ia;
  *qacc = (int32_t)qa;
}

/* doPrepIF (acquisition.cpp:191-236) for ms = 1, 10 or 310: row j*ms + m of the
 * store is the forward FFT of ms block m mixed by the (-fif - 250 j) wipe-off.
 * The wipe-off tables hold 10 ms and repeat (memcpy x 31, :131-137), so sample
 * n of the buffer uses wipe entry n % 20480.  Rows >= 4*ms are NOT written:
 * they keep whatever an earlier, longer prep left (the object's member). */
void sdro_prep_rows(const sdro_cpx *buff, int ms, double fif, int saturate, sdro_cpx *rows)
{
  sdro_cpx *wipe = (sdro_cpx *)malloc(sizeof(sdro_cpx) * SDRO_WIPE);
  sdro_mix w[SDRO_N / 2], iw[SDRO_N / 2];
  static const int32_t r1[16] = {0};
  sdro_twiddles(SDRO_N, w, iw);
  for (int j = 0; j < 4; j++) {
    sdro_sine_gen(wipe, -fif - 250.0 * j, SDRO_FS, SDRO_WIPE);
    for (int m = 0; m < ms; m++) {
      const int off = (m * SDRO_N) % SDRO_WIPE;
      sdro_cpx *dst = rows + (size_t)(j * ms + m) * SDRO_N;
      sdro_cmulsc(buff + (size_t)m * SDRO_N, wipe + off, dst, SDRO_N, 14, saturate);
      sdro_fft(dst, SDRO_N, w, r1);
    }
  }
  free(wipe);
}

/* post-correlation DFT of one delay column: 10 coherent 1-ms values against the
 * 10 dft_rows (wipeoff_gen at lcv*25 - 112.5 Hz, acquisition.cpp:119-120), each
 * sum >> 16 stored as int16 (:364-373), then x86_cmag (int32 wrap) */
static void post_dft(const sdro_cpx *coh, int col, sdro_mix dft[10][10], int32_t pw[10])
{
  sdro_cpx d[10];
  for (int m = 0; m < 10; m++) d[m] = coh[(size_t)m * SDRO_N + col];
  for (int j = 0; j < 10; j++) {
    int32_t ia, qa;
    sdro_cacc(d, dft[j], 10, &ia, &qa);
    const int16_t ti = (int16_t)(ia >> 16), tq = (int16_t)(qa >> 16);
    pw[j] = (int32_t)((uint32_t)(ti * ti) + (uint32_t)(tq * tq));
  }
}

/* first index of the strict maximum, running start 0 (x86_max, x86.cpp:274-293) */
static void max_first(const int32_t *a, int n, int32_t *index, int32_t *mag)
{
  int32_t best = 0, idx = 0;
  for (int k = 0; k < n; k++)
    if (a[k] > best) { best = a[k]; idx = k; }
  *index = idx;
  *mag = best;
}

static void coherent_10(const sdro_cpx *rows, int row0, int lcv, const sdro_cpx *code, int shift,
                        int saturate, const sdro_mix *iw, sdro_cpx *coh)
{
  static const int32_t r2[16] = {0, 0, 0, 0, 0, 0, 0, 1, 0, 1, 0, 1, 1, 1, 1, 1};
  sdro_cpx sh[SDRO_N];
  for (int m = 0; m < 10; m++) {
    const sdro_cpx *row = rows + (size_t)(row0 + m) * SDRO_N;
    for (int k = 0; k < SDRO_N; k++) sh[k] = row[(k + lcv + SDRO_N) & (SDRO_N - 1)];
    sdro_cmulsc(sh, code, coh + (size_t)m * SDRO_N, SDRO_N, shift, saturate);
    sdro_fft(coh + (size_t)m * SDRO_N, SDRO_N, iw, r2);
  }
}

sdro_result sdro_acq_medium(const sdro_cpx *rows, const sdro_cpx *code, int sv, int doppmin,
                            int doppmax, int saturate)
{
  sdro_mix w[SDRO_N / 2], iw[SDRO_N / 2], dft[10][10];
  sdro_twiddles(SDRO_N, w, iw);
  for (int j = 0; j < 10; j++) sdro_wipeoff_gen(dft[j], (float)j * 25.0 - 112.5, 1000.0, 10);
  sdro_cpx *coh = (sdro_cpx *)malloc(sizeof(sdro_cpx) * 10 * SDRO_N);
  int32_t *power = (int32_t *)malloc(sizeof(int32_t) * 10 * SDRO_N);
  sdro_result r;
  memset(&r, 0, sizeof r);
  r.sv = sv;
  int32_t mag = 0;
  const int lmin = doppmin / 1000;
  for (int lcv = lmin; lcv <= doppmax / 1000; lcv++)      /* inclusive, :324 */
    for (int lcv2 = 0; lcv2 < 4; lcv2++) {
      /* baseband_rows[lcv2*20 + lcv3 + k*10] with k = 0 (:341): a 20-row stride
       * over a 10-ms prep, so lcv2 = 1 reads the 500 Hz rows and lcv2 >= 2 reads
       * rows 40..79, which this prep did not write */
      coherent_10(rows, lcv2 * 20, lcv, code, 10, saturate, iw, coh);
      int32_t pw[10];
      for (int c = 0; c < SDRO_N; c++) {
        post_dft(coh, c, dft, pw);
        for (int j = 0; j < 10; j++) power[j * SDRO_N + c] = pw[j];
      }
      int32_t idx, m;
      max_first(power, 10 * SDRO_N, &idx, &m);
      if (m > mag) {
        mag = m;
        r.code_phase = idx % SDRO_N;
        r.doppler = (int32_t)((lcv * 1000) + (lcv2 * 250) + (idx / SDRO_N) * 25.0);
        r.magnitude = (uint32_t)m;
        r.row = (lcv - lmin) * 4 + lcv2;
      }
    }
  r.success = r.magnitude > 0;   /* THRESH_MEDIUM = 0 (config.h:73) */
  free(coh);
  free(power);
  return r;
}

int sdro_weak_shift(int i, int lcv, int lcv2)
{
  /* acquisition.cpp:483-489 */
  const double doppler = (double)(lcv * 1000) + (float)(lcv2 * 250);
  const double code_doppler = (double)i * .02 * 2048000 * doppler / 1.57542e9;
  return (int)floor(code_doppler);
}

sdro_result sdro_acq_weak(const sdro_cpx *rows, const sdro_cpx *code, int sv, int doppmin,
                          int doppmax, int saturate)
{
  sdro_mix w[SDRO_N / 2], iw[SDRO_N / 2], dft[10][10];
  sdro_twiddles(SDRO_N, w, iw);
  for (int j = 0; j < 10; j++) sdro_wipeoff_gen(dft[j], (float)j * 25.0 - 112.5, 1000.0, 10);
  sdro_cpx *coh = (sdro_cpx *)malloc(sizeof(sdro_cpx) * 10 * SDRO_N);
  uint32_t *power = (uint32_t *)malloc(sizeof(uint32_t) * 10 * SDRO_N);
  sdro_result r;
  memset(&r, 0, sizeof r);
  r.sv = sv;
  int32_t mag = 0;
  const int lmin = doppmin / 1000;
  for (int lcv = lmin; lcv < doppmax / 1000; lcv++)       /* exclusive, :452 */
    for (int lcv2 = 0; lcv2 < 4; lcv2++)
      for (int k = 0; k < 2; k++) {
        memset(power, 0, sizeof(uint32_t) * 10 * SDRO_N);
        for (int i = 0; i < 15; i++) {
          coherent_10(rows, lcv2 * 310 + i * 20 + k * 10, lcv, code, 9, saturate, iw, coh);
          const int shift = sdro_weak_shift(i, lcv, lcv2);
          int32_t pw[10];
          for (int c = 0; c < SDRO_N; c++) {
            post_dft(coh, c, dft, pw);
            const int dst = (c + shift + SDRO_N) % SDRO_N;
            for (int j = 0; j < 10; j++) power[j * SDRO_N + dst] += (uint32_t)pw[j];
          }
        }
        int32_t idx, m;
        max_first((const int32_t *)power, 10 * SDRO_N, &idx, &m);
        if (m > mag) {
          mag = m;
          r.code_phase = idx % SDRO_N;
          r.doppler = (int32_t)((lcv * 1000) + (lcv2 * 250) + (idx / SDRO_N) * 25.0);
          r.magnitude = (uint32_t)m;
          r.row = ((lcv - lmin) * 4 + lcv2) * 2 + k;
        }
      }
  r.success = r.magnitude > 0;   /* THRESH_WEAK = 0 (config.h:74) */
  free(coh);
  free(power);
  return r;
}

/* ---- PRN_Codes (gen_fft_codes.m with prn_gen.m) ------------------------ */
static const int k_g2_delay[51] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256,
                                   257, 258, 469, 470, 471, 472, 473, 474, 509, 512, 513, 514,
                                   515, 516, 859, 860, 861, 862, 145, 175, 52, 21, 237, 235, 886,
                                   657, 634, 762, 355, 1012, 176, 603, 130, 359, 595, 68, 386};

static void fft_d(double *re, double *im, int n)
{
  const int m = ilog2(n);
  for (int k = 0; k < n; k++) {
    const int j = bitrev(k, m);
    if (j > k) {
      double t = re[k]; re[k] = re[j]; re[j] = t;
      t = im[k]; im[k] = im[j]; im[j] = t;
    }
  }
  for (int len = 2; len <= n; len <<= 1) {
    for (int j = 0; j < len / 2; j++) {
      const double ang = -2.0 * M_PI * j / len, wr = cos(ang), wi = sin(ang);
      for (int s = 0; s < n; s += len) {
        const int a = s + j, b = a + len / 2;
        const double xr = re[b] * wr - im[b] * wi, xi = re[b] * wi + im[b] * wr;
        re[b] = re[a] - xr; im[b] = im[a] - xi;
        re[a] += xr; im[a] += xi;
      }
    }
  }
}

static double round_away(double v) { return v < 0 ? -floor(-v + 0.5) : floor(v + 0.5); }

void sdro_prn_codes(int16_t *out /* [51][2048][2] */)
{
  int g1[1023], g2[1023], r1[10], r2[10];
  for (int k = 0; k < 10; k++) r1[k] = r2[k] = 1;
  for (int k = 0; k < 1023; k++) {
    g1[k] = r1[0];
    g2[k] = r2[0];
    const int f1 = r1[7] ^ r1[0];
    const int f2 = (r2[8] + r2[7] + r2[4] + r2[2] + r2[1] + r2[0]) & 1;
    memmove(r1, r1 + 1, 9 * sizeof(int));
    memmove(r2, r2 + 1, 9 * sizeof(int));
    r1[9] = f1;
    r2[9] = f2;
  }
  int idx[SDRO_N];
  for (int k = 0; k < SDRO_N; k++) idx[k] = (int)round_away(1.0 + (k * 1022.0) / (SDRO_N - 1)) - 1;
  double *re = (double *)malloc(sizeof(double) * 51 * SDRO_N);
  double *im = (double *)malloc(sizeof(double) * 51 * SDRO_N);
  double amax = 0;
  for (int p = 0; p < 51; p++) {
    const int d = 1023 - k_g2_delay[p];
    double *R = re + (size_t)p * SDRO_N, *I = im + (size_t)p * SDRO_N;
    for (int k = 0; k < SDRO_N; k++) {
      const int c = idx[k];
      R[k] = 2.0 * (g1[c] ^ g2[(c + d) % 1023]) - 1.0;
      I[k] = 0.0;
    }
    fft_d(R, I, SDRO_N);
    for (int k = 0; k < SDRO_N; k++) {
      I[k] = -I[k];                                    /* conj */
      const double a = hypot(R[k], I[k]);
      if (a > amax) amax = a;
    }
  }
  const double scale = 512.0 / amax;
  for (size_t k = 0; k < (size_t)51 * SDRO_N; k++) {
    out[2 * k] = (int16_t)round_away(re[k] * scale);
    out[2 * k + 1] = (int16_t)round_away(im[k] * scale);
  }
  free(re);
  free(im);
}
