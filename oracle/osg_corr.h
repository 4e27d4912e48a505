/*
 * oracle/osg_corr.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the OSGPS software GP2021 correlator
 * (reference: osgnss_next_step/src/correlator/correlator.c).  Used as the
 * parity checker for the HIP tracking kernel and as the `cpu_baseline`
 * ("port") leg of bench.py.  The product path never links this.
 *
 * Parity pinned: tests/test_oracle_osg.py checks this restatement bit-exact
 * against oracle/_ref/libosg_ref.so (the reference compiled from its own
 * sources) and against the committed fixtures in tests/golden/.
 */
#ifndef ORACLE_OSG_CORR_H
#define ORACLE_OSG_CORR_H
#include <stdint.h>

#define OSGO_MAX_CH 16

/* One emulated GP2021 correlator instance (the reference keeps these as file
 * statics / globals, correlator.c:25-47; here they live in a struct). */
typedef struct {
  int      n_channels;          /* N_CHANNELS (globals.h:7)               */
  int      use_iq;              /* use_iq_processing (globals.h:56)        */
  int64_t  tic, tic_ref;        /* correlator.c:30                          */
  int      ms_counter[OSGO_MAX_CH], bit_counter[OSGO_MAX_CH];
  /* struct gp2021_channel (correlator.c:36-47) */
  uint32_t carrier_phase[OSGO_MAX_CH], carrier_cycle[OSGO_MAX_CH], code_phase[OSGO_MAX_CH];
  uint16_t half_chip[OSGO_MAX_CH];
  int32_t  acc[OSGO_MAX_CH][6];  /* REG_read order: IL, QL, IP, QP, IE, QE */
  int32_t  reg_read[256], reg_write[256];
} osgo_t;

/* Size in bytes of the flat E/P/L table image (see osg_corr.c). */
int  osgo_table_bytes(void);
/* Copy the flat table image (late | pad | prompt | pad | early | zeros). */
void osgo_table_image(int8_t *out);

void osgo_init(osgo_t *o, int n_channels, int use_iq, double samp_rate, double tic_period);
void osgo_sim(osgo_t *o, const int8_t *IF, long nsamp);
/* Test-only: log every dump of later osgo_sim calls into buf (cap entries of 7
 * int32 {ch, IL, QL, IP, QP, IE, QE}); NULL stops logging.  Not thread-safe. */
void osgo_dump_log(int32_t *buf, int cap);
int  osgo_dump_count(void);

/* Register accessors mirroring gp2021/gp2021.c:11-130 (host side). */
void osgo_ch_cntl(osgo_t *o, int ch, int prn);
void osgo_ch_carrier(osgo_t *o, int ch, long freq);
void osgo_ch_code(osgo_t *o, int ch, long freq);
void osgo_ch_code_slew(osgo_t *o, int ch, int slew);
void osgo_ch_epoch_load(osgo_t *o, int ch, unsigned data);
int  osgo_reg_read(const osgo_t *o, int addr);   /* from_gps: truncates to short */

/* Multi-threaded CPU baseline: run `n_inst` independent correlator instances
 * (each n_channels on its own IF stream of if_calls*nsamp complex samples,
 * replayed cyclically) for n_calls calls on `threads` pthreads.  Returns the
 * total channel-samples processed. */
double osgo_bench(int n_inst, int n_channels, const int8_t *IF, long nsamp, int n_calls,
                  int if_calls, long carrier_freq, long code_freq, int threads);

int  osgo_sizeof(void);
#endif
