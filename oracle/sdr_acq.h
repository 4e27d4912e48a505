/*
 * oracle/sdr_acq.h -- TEST INFRASTRUCTURE ONLY (see sdr_acq.c).
 * CPU restatement of the GPS-SDR int16 strong acquisition.
 */
#ifndef ORACLE_SDR_ACQ_H
#define ORACLE_SDR_ACQ_H
#include <stdint.h>

#define SDRO_N 2048            /* SAMPS_MS, defines.h:150 */
#define SDRO_FS 2048000.0      /* SAMPLE_FREQUENCY, defines.h:151 */
#define SDRO_WIPE 20480        /* 10 ms wipe-off tables (acquisition.cpp:123-128) */
#define SDRO_ROWS 1240         /* baseband_rows: 4 x 310 (acquisition.cpp:107-110) */

typedef struct { int16_t i, q; } sdro_cpx;             /* CPX, sdr_structs.h:34-38 */
typedef struct { int16_t i, nq, q, ni; } sdro_mix;     /* MIX, sdr_structs.h:53-60 */

typedef struct {               /* the result fields of Acq_Command_S (structs.h:130-164) */
  int32_t sv, code_phase, doppler;
  uint32_t magnitude;
  int32_t success, row;        /* row: (lcv - doppmin/1000)*4 + lcv2 of the winner */
} sdro_result;

void sdro_sine_gen(sdro_cpx *dst, double f, double fs, int n);
void sdro_twiddles(int n, sdro_mix *w, sdro_mix *iw);
void sdro_fft(sdro_cpx *x, int n, const sdro_mix *w, const int32_t *rank_scale);
void sdro_cmulsc(const sdro_cpx *a, const sdro_cpx *b, sdro_cpx *c, int n, int shift, int saturate);
void sdro_cmag_max(const sdro_cpx *a, int n, int32_t *index, int32_t *mag);
void sdro_prep_if(const sdro_cpx *buff, double fif, int saturate, sdro_cpx rows[4][SDRO_N]);
sdro_result sdro_acq_strong(sdro_cpx rows[4][SDRO_N], const sdro_cpx *code, int sv, int doppmin,
                            int doppmax, int saturate);
void sdro_prn_codes(int16_t *out);
void sdro_wipeoff_gen(sdro_mix *dst, double f, double fs, int n);
void sdro_cacc(const sdro_cpx *a, const sdro_mix *b, int n, int32_t *iacc, int32_t *qacc);
void sdro_prep_rows(const sdro_cpx *buff, int ms, double fif, int saturate, sdro_cpx *rows);
int sdro_weak_shift(int i, int lcv, int lcv2);
/* row: medium (lcv-lmin)*4 + lcv2; weak ((lcv-lmin)*4 + lcv2)*2 + k */
sdro_result sdro_acq_medium(const sdro_cpx *rows, const sdro_cpx *code, int sv, int doppmin,
                            int doppmax, int saturate);
sdro_result sdro_acq_weak(const sdro_cpx *rows, const sdro_cpx *code, int sv, int doppmin,
                          int doppmax, int saturate);
#endif
