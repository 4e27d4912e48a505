/*
 * oracle/e2e_receiver.c -- end-to-end drop-in harness (BASELINE config 1/3).
 *
 * The main loop of osgnss_next_step/src/osgnss_next_step.c:168-184 without
 * the Windows console (display.c) and the hard-coded e:\ debug path:
 *   init_tracking_loops_parameter -> correlator_init(tic_period) ->
 *   channel allocation -> while(fread 512 us of IQ) { Sim_GP2021_int; gpsisr; }
 *
 * It is linked twice by oracle/Makefile, with the reference's own
 * gp2021/gp2021.c and isr/osgpsisr.c (compiled unmodified from
 * /root/reference) in both:
 *   _ref/e2e_ref : + reference correlator/correlator.c   (CPU)
 *   _ref/e2e_gpu : + libgnsscorr.so (correlator_init, Sim_GP2021_int,
 *                    REG_read/REG_write on the MI355X)
 * and writes a per-call trace (REG_read words, loop state of every channel).
 * The two traces must be byte-identical: the closed-loop DLL/PLL sees exactly
 * the same accumulators from the GPU as from the reference correlator.
 *
 * The _16368 builds (oracle/Makefile e2e16368) stream globals.h with SAMP_RATE
 * rewritten to 16.368e6 into every compile (BASELINE config 1); e2e_gpu_16368
 * runs with GNSSCORR_SAMP_RATE=16.368e6 for the shim's correlator_init.
 *
 * usage: e2e_xxx <if.bin> <trace.bin> <n_calls> <prn ch0> [prn ch1 ...]
 */
#ifndef MAIN
#define MAIN
#endif
#include "globals.h"
#include <stdlib.h>
#include <string.h>

extern int REG_read[256], REG_write[256];
void correlator_init(double tic_period);
void Sim_GP2021_int(char *IF, long nsamp);
void gpsisr(void);
void ch_cntl(int, int);
void ch_carrier(int, long);
void ch_code(int, long);
void calc_FLL_assisted_PLL_filter_loop_coefs(long, long, long, double *, double *, double *);
void convert_FLL_assisted_PLL_loop_filter_coefs_to_integer(double, double, double, int *, int *, int *);
void calc_DLL_loop_filter_coefs(long, long, double *, double *);
void convert_DLL_loop_filter_coefs_to_integer(double, double, int *, int *);

/* osgnss_next_step.c:73-84 (reset_all_correlator_channles) */
static void reset_channels(void)
{
  for (int ch = 0; ch < N_CHANNELS; ch++) {
    ch_cntl(ch, 0);
    ch_carrier(ch, gps_carrier_ref);
    ch_code(ch, gps_code_ref);
    chan[ch].state = CHANNEL_ACQUISITION;
    chan[ch].carrier_cold_corr = 0;
    chan[ch].del_freq = 1;
    chan[ch].n_freq = 0;
    chan[ch].search_max_PRN_delay = 2045;
    chan[ch].search_max_f = 5;
    chan[ch].ms_set = 0;
  }
}

/* one trace record per call */
typedef struct {
  int32_t reg_read[256];
  int32_t state[N_CHANNELS];
  int64_t carr_freq[N_CHANNELS];
  int64_t code_freq[N_CHANNELS];
  int32_t n_freq[N_CHANNELS];
  int32_t codes[N_CHANNELS];
} trace_t;

int main(int argc, char **argv)
{
  if (argc < 5) {
    fprintf(stderr, "usage: %s if.bin trace.bin n_calls prn0 [prn1 ...]\n", argv[0]);
    return 2;
  }
  FILE *fin = fopen(argv[1], "rb"), *fout = fopen(argv[2], "wb");
  if (!fin || !fout) { perror("open"); return 2; }
  const long n_calls = atol(argv[3]);
  corr_out = fopen("/dev/null", "w");     /* osgpsisr.c DEBUG_TRACKING sink */

  /* osgnss_next_step.c:99-107 (init_tracking_loops_parameter) */
  calc_FLL_assisted_PLL_filter_loop_coefs(Bnp, Bnf, FLL_a_PLL_integ_time, &FLL_a_PLL_k1,
                                          &FLL_a_PLL_k2, &FLL_a_PLL_k3);
  convert_FLL_assisted_PLL_loop_filter_coefs_to_integer(FLL_a_PLL_k1, FLL_a_PLL_k2, FLL_a_PLL_k3,
                                                        &FLL_a_PLL_i1, &FLL_a_PLL_i2, &FLL_a_PLL_i3);
  calc_DLL_loop_filter_coefs(Bnd, DLL_integ_time, &DLL_k1, &DLL_k2);
  convert_DLL_loop_filter_coefs_to_integer(DLL_k1, DLL_k2, &DLL_i1, &DLL_i2);

  correlator_init(tic_period);
  const long nsamp = (long)(SAMP_RATE * interr_int / 1.0e6);   /* :442 */
  reset_channels();
  for (int i = 4; i < argc && i - 4 < N_CHANNELS; i++) ch_cntl(i - 4, atoi(argv[i]));

  char *IF = (char *)malloc((size_t)nsamp * 2);
  trace_t tr;
  for (long k = 0; k < n_calls; k++) {
    if (fread(IF, 1, (size_t)nsamp * 2, fin) != (size_t)nsamp * 2) break;
    Sim_GP2021_int(IF, nsamp);
    gpsisr();
    memcpy(tr.reg_read, REG_read, sizeof tr.reg_read);
    for (int ch = 0; ch < N_CHANNELS; ch++) {
      tr.state[ch] = chan[ch].state;
      tr.carr_freq[ch] = chan[ch].carrier_freq + chan[ch].carrFreq;
      tr.code_freq[ch] = chan[ch].codeFreq;
      tr.n_freq[ch] = chan[ch].n_freq;
      tr.codes[ch] = chan[ch].codes;
    }
    fwrite(&tr, sizeof tr, 1, fout);
  }
  fclose(fout);
  free(IF);
  return 0;
}
