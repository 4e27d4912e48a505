/*
 * sdr_host.c -- host-side tables of the GPS-SDR integer acquisition
 * (REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER, "SDR/").
 *
 *  gnsscorr_sdr_sine_gen   SDR/accessories/misc.cpp:95-115: Q14-ish wipe-off
 *                          floor(16383*cos(phase)) with a float phase accumulator
 *                          and the C++ float overloads cos(float)/sin(float)
 *  gnsscorr_sdr_twiddles   SDR/objects/fft.cpp:114-147: floor(16384*cos/sin)
 *  gnsscorr_sdr_post_dft   the 10 x 10 post-correlation DFT rows of the medium /
 *                          weak acquisition: wipeoff_gen (misc.cpp:148-168, fp64
 *                          phase) at lcv*25 - 112.5 Hz, fs 1 kHz
 *                          (acquisition.cpp:119-120)
 *  gnsscorr_sdr_prn_codes  SDR/accessories/gen_fft_codes.m + prn_gen.m: the
 *                          PRN_Codes table (conj FFT of the 2.048 Msps resampled
 *                          C/A code, scaled to 9 bits, rounded half away from 0)
 * These run once per context; the GPU kernels use them as uploaded tables.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "gnsscorr_internal.h"

#define SDR_N 2048

void gnsscorr_sdr_sine_gen(int16_t *out, double f, double fs, int n)
{
  float ph = 0.0f;
  const float step = (float)6.283185307179586 * f / fs;
  for (int k = 0; k < n; k++, ph += step) {
    out[2 * k] = (int16_t)floor(16383.0 * (double)cosf(ph));
    out[2 * k + 1] = (int16_t)floor(16383.0 * (double)sinf(ph));
  }
}

void gnsscorr_sdr_twiddles(int16_t *w, int16_t *iw)
{
  const double pi = 3.14159265358979323846264338327;
  for (int k = 0; k < SDR_N / 2; k++) {
    const double ph = (-2 * pi * k) / SDR_N;
    const double c = floor(16384 * cos(ph)), s = floor(16384 * sin(ph));
    w[2 * k] = (int16_t)c;
    w[2 * k + 1] = (int16_t)s;
    iw[2 * k] = (int16_t)c;
    iw[2 * k + 1] = (int16_t)(-s);
  }
}

/* dft[j][m] as two packed int16 pairs per entry: {i, nq} and {q, ni} (MIX,
 * sdr_structs.h:53-60), the operands of the two pmaddwd halves of sse_cacc */
void gnsscorr_sdr_post_dft(int16_t *out /* [10][10][4] */)
{
  for (int j = 0; j < 10; j++) {
    double ph = 0.0;
    const double step = 6.283185307179586 * ((float)j * 25.0 - 112.5) / 1000.0;
    for (int m = 0; m < 10; m++, ph += step) {
      const int16_t c = (int16_t)floor(16383.0 * cos(ph)), s = (int16_t)floor(16383.0 * sin(ph));
      int16_t *o = out + 4 * (j * 10 + m);
      o[0] = c;
      o[1] = (int16_t)(-s);
      o[2] = s;
      o[3] = c;
    }
  }
}

/* in-place radix-2 FFT in double, natural order in and out */
static void dfft(double *re, double *im, int n, int logn)
{
  for (int k = 0; k < n; k++) {
    int r = 0;
    for (int b = 0; b < logn; b++) r |= ((k >> b) & 1) << (logn - 1 - b);
    if (r > k) {
      double t = re[k]; re[k] = re[r]; re[r] = t;
      t = im[k]; im[k] = im[r]; im[r] = t;
    }
  }
  for (int h = 1; h < n; h <<= 1) {
    for (int j = 0; j < h; j++) {
      const double a = -M_PI * j / h, c = cos(a), s = sin(a);
      for (int base = 0; base < n; base += 2 * h) {
        double *ar = re + base + j, *ai = im + base + j;
        const double br = ar[h] * c - ai[h] * s, bi = ar[h] * s + ai[h] * c;
        ar[h] = ar[0] - br; ai[h] = ai[0] - bi;
        ar[0] += br; ai[0] += bi;
      }
    }
  }
}

static double rnd_away(double v) { return v < 0 ? -floor(0.5 - v) : floor(v + 0.5); }

int gnsscorr_sdr_prn_codes(int16_t *out)
{
  static const short g2d[51] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257,
                                258, 469, 470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516,
                                859, 860, 861, 862, 145, 175, 52, 21, 237, 235, 886, 657, 634,
                                762, 355, 1012, 176, 603, 130, 359, 595, 68, 386};
  if (!out) return GNSSCORR_EINVAL;
  /* G1 / G2 sequences from all-ones registers (prn_gen.m) as bit-shift LFSRs */
  uint8_t g1[1023], g2[1023];
  unsigned s1 = 0x3FF, s2 = 0x3FF;   /* bit b = register stage b (stage 0 is output) */
  for (int k = 0; k < 1023; k++) {
    g1[k] = s1 & 1u;
    g2[k] = s2 & 1u;
    const unsigned f1 = ((s1 >> 7) ^ s1) & 1u;
    const unsigned f2 = ((s2 >> 8) ^ (s2 >> 7) ^ (s2 >> 4) ^ (s2 >> 2) ^ (s2 >> 1) ^ s2) & 1u;
    s1 = (s1 >> 1) | (f1 << 9);
    s2 = (s2 >> 1) | (f2 << 9);
  }
  double *re = (double *)malloc(sizeof(double) * 51 * SDR_N);
  double *im = (double *)calloc((size_t)51 * SDR_N, sizeof(double));
  if (!re || !im) { free(re); free(im); return GNSSCORR_ENOMEM; }
  double peak = 0;
  for (int p = 0; p < 51; p++) {
    double *R = re + (size_t)p * SDR_N, *I = im + (size_t)p * SDR_N;
    const int d = 1023 - g2d[p];
    for (int k = 0; k < SDR_N; k++) {
      /* resample: round(linspace(1, 1023, 2048)) (1-based chip index) */
      const int chip = (int)rnd_away(1.0 + (k * 1022.0) / (SDR_N - 1)) - 1;
      R[k] = (g1[chip] ^ g2[(chip + d) % 1023]) ? 1.0 : -1.0;
    }
    dfft(R, I, SDR_N, 11);
    for (int k = 0; k < SDR_N; k++) {
      I[k] = -I[k];
      const double m = hypot(R[k], I[k]);
      if (m > peak) peak = m;
    }
  }
  const double scale = 512.0 / peak;
  for (size_t k = 0; k < (size_t)51 * SDR_N; k++) {
    out[2 * k] = (int16_t)rnd_away(re[k] * scale);
    out[2 * k + 1] = (int16_t)rnd_away(im[k] * scale);
  }
  free(re);
  free(im);
  return GNSSCORR_OK;
}

/* code_gen (SDR/accessories/misc.cpp:28-87): 0/1 chips of the 0-based G2-delay
 * index sv (G1 xor G2 delayed by 1023 - delay[sv]). */
void gnsscorr_sdr_code_gen(int sv, uint8_t *chips)
{
  static const short g2d[51] = {5, 6, 7, 8, 17, 18, 139, 140, 141, 251, 252, 254, 255, 256, 257,
                                258, 469, 470, 471, 472, 473, 474, 509, 512, 513, 514, 515, 516,
                                859, 860, 861, 862, 145, 175, 52, 21, 237, 235, 886, 657, 634,
                                762, 355, 1012, 176, 603, 130, 359, 595, 68, 386};
  uint8_t g1[1023], g2[1023];
  unsigned s1 = 0x3FF, s2 = 0x3FF;
  for (int k = 0; k < 1023; k++) {
    g1[k] = s1 & 1u;
    g2[k] = s2 & 1u;
    const unsigned f1 = ((s1 >> 7) ^ s1) & 1u;
    const unsigned f2 = ((s2 >> 8) ^ (s2 >> 7) ^ (s2 >> 4) ^ (s2 >> 2) ^ (s2 >> 1) ^ s2) & 1u;
    s1 = (s1 >> 1) | (f1 << 9);
    s2 = (s2 >> 1) | (f2 << 9);
  }
  const int d = 1023 - g2d[sv];
  for (int k = 0; k < 1023; k++) chips[k] = g1[k] ^ g2[(k + d) % 1023];
}

/* GN3S front-end products (SDR/objects/gps_source.cpp:92-93, :733-738): for
 * each 2-bit code l (LUT {-3,-1,1,3}) and NCO index p, the int16 values the
 * reference stores, (int16)(LUT[l] * (+8 cos(2 pi p/1024))) as I and
 * (int16)(LUT[l] * (-8 sin(2 pi p/1024))) as Q (double product, truncation).
 * out[(l * 1024 + p) * 2 + {0, 1}] = {I, Q}. */
void gnsscorr_sdr_gn3s_products(int16_t *out)
{
  static const int16_t lut[4] = {-3, -1, 1, 3};
  for (int p = 0; p < 1024; p++) {
    const double s = -8 * sin(2 * M_PI * p / 1024);
    const double c = +8 * cos(2 * M_PI * p / 1024);
    for (int l = 0; l < 4; l++) {
      out[(l * 1024 + p) * 2 + 0] = (int16_t)(lut[l] * c);
      out[(l * 1024 + p) * 2 + 1] = (int16_t)(lut[l] * s);
    }
  }
}
