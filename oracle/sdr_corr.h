/*
 * oracle/sdr_corr.h -- TEST INFRASTRUCTURE ONLY (see sdr_corr.c).
 * CPU restatement of the GPS-SDR tracking correlator (Correlator class).
 */
#ifndef ORACLE_SDR_CORR_H
#define ORACLE_SDR_CORR_H
#include <stdint.h>
#include "sdr_acq.h"

#define SDRC_N 2048                 /* SAMPS_MS: one packet            */
#define SDRC_ROW (2 * SDRC_N)       /* pre-sampled row length          */
#define SDRC_IF 38400               /* IF_FREQUENCY (signaldef.h:34)   */
#define SDRC_CARRIER_SPACING 10     /* config.h:82                     */
#define SDRC_CARRIER_BINS 1500      /* MAX_DOPPLER_ABSOLUTE / spacing  */
#define SDRC_SBINS (2 * SDRC_CARRIER_BINS + 1)
#define SDRC_CODE_BINS 50           /* config.h:81                     */
#define SDRC_CBINS (2 * SDRC_CODE_BINS + 1)

typedef sdro_cpx sdrc_cpx;

typedef struct {                    /* Correlator_State_S (sdr_structs.h:141-168), pointers as offsets */
  double code_phase, carrier_phase, carrier_phase_prev, code_phase_mod, carrier_phase_mod;
  double code_nco, carrier_nco;
  uint32_t chan, sv, navigate, active, count, scount;
  uint32_t _1ms_epoch, _20ms_epoch, _z_count, rollover;
  uint32_t cbin[3], sbin;
  int32_t coff[3], soff;            /* pcode[k] - code_rows[cbin[k]], psine - sine row */
} sdrc_state;

typedef struct { int32_t I[3], Q[3]; } sdrc_corr;      /* Correlation_S */

typedef struct {                    /* NCO_Command_S (sdr_structs.h:112-125) */
  double carrier_nco, code_nco;
  uint32_t kill, reset_1ms, reset_20ms, set_z_count, z_count, length, navigate, pad;
} sdrc_feedback;

typedef struct { const sdrc_cpx *carrier; const int8_t *code; } sdrc_tables_t;

typedef void (*sdrc_cb)(void *user, int ch, const sdrc_state *s, const sdrc_corr *c,
                        sdrc_feedback *f);

void sdrc_code_gen(int sv, uint8_t *chips);
void sdrc_tables(sdrc_cpx *carrier, int8_t *code);
void sdrc_accum(const sdrc_cpx *data, const sdrc_cpx *sine, const int8_t *e, const int8_t *p,
                const int8_t *l, int samps, int saturate, sdrc_corr *c);
void sdrc_update(sdrc_state *s, int32_t samps);
void sdrc_rotate(sdrc_state *s, sdrc_corr *c);
void sdrc_feedback_apply(sdrc_state *s, const sdrc_feedback *f);
void sdrc_rebin(sdrc_state *s);
void sdrc_correlate(const sdrc_tables_t *t, const sdrc_cpx *packet, int n_ch, sdrc_state *st,
                    sdrc_corr *corr, int saturate, sdrc_cb cb, void *user);
void sdrc_init_chan(sdrc_state *s, int sv, int acq_code_phase, int acq_doppler,
                    double packets_since_acq);
void sdrc_test_loop(void *user, int ch, const sdrc_state *s, const sdrc_corr *c,
                    sdrc_feedback *f);
#endif
