/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * Host-side glue that lets the UNMODIFIED reference OSGPS correlator
 * (osgnss_next_step/src/correlator/correlator.c + gp2021/gp2021.c +
 *  isr/osgpsisr.c, compiled by oracle/Makefile straight from /root/reference
 *  into oracle/_ref/) be driven from Python (ctypes) to produce golden vectors.
 *
 * The reference keeps its receiver globals in include/globals.h behind
 * `#define MAIN` (osgnss_next_step.c:1-2 of the main program defines them);
 * this file plays the role of that main translation unit so the reference
 * objects link, and adds two tiny accessors.
 */
#define MAIN
#include <stdint.h>
#include <string.h>
#include "globals.h"

/* correlator.h defines these as tentative definitions (needs -fcommon). */
extern int REG_read[256], REG_write[256];

/* osgpsisr.c writes DEBUG_TRACKING vectors to corr_out; point it at /dev/null
 * so the end-to-end receiver harness can run the unmodified ISR. */
void ref_harness_open_debug(void)
{
  if (!corr_out) corr_out = fopen("/dev/null", "w");
}

/* Byte size of the reference's tracking_channel struct (structs.h:86-128), so
 * Python can walk chan[] without restating the layout. */
int ref_harness_sizeof_tracking_channel(void) { return (int)sizeof(tracking_channel); }

/* ---- gpsisr driver (osgpsisr.c:360-404) for the GPU channel-loop tests ----
 * The flat loop record mirrors gnsscorr_osg_loop (include/gnsscorr.h); these
 * accessors copy it to / from the reference's tracking_channel chan[ch], set
 * the REG_read words gpsisr reads, run the UNMODIFIED gpsisr once and return
 * the REG_write words it wrote. */
typedef struct {
  int32_t state, n_freq, i_confirm, n_thresh, codes, del_freq;
  int32_t sign_pos, prev_sign_pos, sign_count, ms_count, ms_set;
  int32_t search_max_prn_delay, search_max_f, cn0, bit, exited;
  int16_t accum[6], prev_accum[6];
  int64_t early_mag, prompt_mag, late_mag;
  int64_t cross, dot, carr_error, old_carr_error, freq_error;
  int64_t carr_nco, old_carr_nco, carr_freq, carr_freq_basis;
  int64_t code_error, old_code_error, code_freq, code_freq_basis, code_nco, old_code_nco;
  int64_t ch_time, carrier_freq, carrier_cold_corr;
  uint64_t ms_sign;
} flat_loop;

static void acc_to(const accum *a, int16_t *o)
{
  o[0] = a->i_prompt; o[1] = a->q_prompt; o[2] = a->i_late;
  o[3] = a->q_late; o[4] = a->i_early; o[5] = a->q_early;
}
static void acc_from(const int16_t *o, accum *a)
{
  a->i_prompt = o[0]; a->q_prompt = o[1]; a->i_late = o[2];
  a->q_late = o[3]; a->i_early = o[4]; a->q_early = o[5];
}

void ref_isr_set_chan(int ch, const flat_loop *f)
{
  tracking_channel *c = &chan[ch];
  c->state = f->state; c->n_freq = f->n_freq; c->i_confirm = f->i_confirm;
  c->n_thresh = f->n_thresh; c->codes = f->codes; c->del_freq = f->del_freq;
  c->sign_pos = f->sign_pos; c->prev_sign_pos = f->prev_sign_pos;
  c->sign_count = f->sign_count; c->ms_count = f->ms_count; c->ms_set = f->ms_set;
  c->search_max_PRN_delay = f->search_max_prn_delay; c->search_max_f = f->search_max_f;
  c->CN0 = (char)f->cn0; c->bit = (char)f->bit;
  acc_from(f->accum, &c->accum); acc_from(f->prev_accum, &c->prev_accum);
  c->accum_mean.early_mag = f->early_mag; c->accum_mean.prompt_mag = f->prompt_mag;
  c->accum_mean.late_mag = f->late_mag;
  c->cross = f->cross; c->dot = f->dot; c->carrError = f->carr_error;
  c->oldCarrError = f->old_carr_error; c->freqError = f->freq_error;
  c->carrNco = f->carr_nco; c->oldCarrNco = f->old_carr_nco; c->carrFreq = f->carr_freq;
  c->carrFreqBasis = f->carr_freq_basis; c->codeError = f->code_error;
  c->oldCodeError = f->old_code_error; c->codeFreq = f->code_freq;
  c->codeFreqBasis = f->code_freq_basis; c->codeNco = f->code_nco;
  c->oldCodeNco = f->old_code_nco; c->ch_time = f->ch_time; c->carrier_freq = f->carrier_freq;
  c->carrier_cold_corr = f->carrier_cold_corr; c->ms_sign = f->ms_sign;
}

void ref_isr_get_chan(int ch, flat_loop *f)
{
  const tracking_channel *c = &chan[ch];
  memset(f, 0, sizeof *f);
  f->state = c->state; f->n_freq = c->n_freq; f->i_confirm = c->i_confirm;
  f->n_thresh = c->n_thresh; f->codes = c->codes; f->del_freq = c->del_freq;
  f->sign_pos = c->sign_pos; f->prev_sign_pos = c->prev_sign_pos;
  f->sign_count = c->sign_count; f->ms_count = c->ms_count; f->ms_set = c->ms_set;
  f->search_max_prn_delay = c->search_max_PRN_delay; f->search_max_f = c->search_max_f;
  f->cn0 = c->CN0; f->bit = c->bit;
  acc_to(&c->accum, f->accum); acc_to(&c->prev_accum, f->prev_accum);
  f->early_mag = c->accum_mean.early_mag; f->prompt_mag = c->accum_mean.prompt_mag;
  f->late_mag = c->accum_mean.late_mag;
  f->cross = c->cross; f->dot = c->dot; f->carr_error = c->carrError;
  f->old_carr_error = c->oldCarrError; f->freq_error = c->freqError;
  f->carr_nco = c->carrNco; f->old_carr_nco = c->oldCarrNco; f->carr_freq = c->carrFreq;
  f->carr_freq_basis = c->carrFreqBasis; f->code_error = c->codeError;
  f->old_code_error = c->oldCodeError; f->code_freq = c->codeFreq;
  f->code_freq_basis = c->codeFreqBasis; f->code_nco = c->codeNco;
  f->old_code_nco = c->oldCodeNco; f->ch_time = c->ch_time; f->carrier_freq = c->carrier_freq;
  f->carrier_cold_corr = c->carrier_cold_corr; f->ms_sign = c->ms_sign;
}

/* loop constants exactly as osgnss_next_step.c:99-107 (init_tracking_loops_parameter) computes them, plus
 * the correlator_init words; out = {i1, i2, i3, dll1, dll2, carrier_ref,
 * code_ref, d_freq} */
void gpsisr(void);
void correlator_init(double tic_period);
void ref_isr_constants(long *out)
{
  calc_FLL_assisted_PLL_filter_loop_coefs(Bnp, Bnf, FLL_a_PLL_integ_time, &FLL_a_PLL_k1,
                                          &FLL_a_PLL_k2, &FLL_a_PLL_k3);
  convert_FLL_assisted_PLL_loop_filter_coefs_to_integer(FLL_a_PLL_k1, FLL_a_PLL_k2, FLL_a_PLL_k3,
                                                        &FLL_a_PLL_i1, &FLL_a_PLL_i2, &FLL_a_PLL_i3);
  calc_DLL_loop_filter_coefs(Bnd, DLL_integ_time, &DLL_k1, &DLL_k2);
  convert_DLL_loop_filter_coefs_to_integer(DLL_k1, DLL_k2, &DLL_i1, &DLL_i2);
  correlator_init(tic_period);
  out[0] = FLL_a_PLL_i1; out[1] = FLL_a_PLL_i2; out[2] = FLL_a_PLL_i3;
  out[3] = DLL_i1; out[4] = DLL_i2;
  out[5] = gps_carrier_ref; out[6] = gps_code_ref; out[7] = d_freq;
}

/* One gpsisr() with REG_read set from dumps[ch][6] (IL QL IP QP IE QE) for the
 * channels in dump_mask; REG_write (256 words) before and after through regs. */
void ref_isr_step(int dump_mask, const int32_t *dumps, int32_t *regs)
{
  if (!corr_out) corr_out = fopen("/dev/null", "w");
  memcpy(REG_write, regs, sizeof(int) * 256);
  for (int ch = 0; ch < N_CHANNELS; ch++)
    for (int k = 0; k < 6; k++) REG_read[(ch << 3) + 0x84 + k] = dumps[ch * 6 + k];
  REG_read[0x82] = dump_mask;
  gpsisr();
  memcpy(regs, REG_write, sizeof(int) * 256);
}

/* ---- CPU baseline: the reference Sim_GP2021_int itself, one core ---------
 * 12 channels active (PRNs 1..12, the given carrier / code words), n_calls
 * calls over if_calls rotating IF buffers of nsamp interleaved int8 I,Q
 * samples.  Returns channel-samples processed.  The reference keeps its state
 * in globals, so this is one instance on one thread by construction. */
void Sim_GP2021_int(char *IF, long nsamp);
void ch_cntl(int ch, int prn);
void ch_carrier(int ch, long freq);
void ch_code(int ch, long freq);
double ref_bench(const int8_t *IF, long nsamp, int n_calls, int if_calls, long carrier_word,
                 long code_word)
{
  use_iq_processing = 1;
  correlator_init(tic_period);
  for (int ch = 0; ch < N_CHANNELS; ch++) {
    ch_cntl(ch, 1 + ch);
    ch_carrier(ch, carrier_word + 13 * ch);
    ch_code(ch, code_word);
  }
  double work = 0;
  for (int c = 0; c < n_calls; c++) {
    Sim_GP2021_int((char *)IF + (size_t)(c % if_calls) * (size_t)nsamp * 2, nsamp);
    work += (double)N_CHANNELS * (double)nsamp;
  }
  return work;
}
