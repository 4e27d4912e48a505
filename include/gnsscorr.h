/*
 * gnsscorr.h -- C ABI of the MI355X-native GNSS correlator (libgnsscorr.so).
 *
 * Two layers:
 *
 *  1. Batched API (gnsscorr_*): explicit contexts, explicit per-channel state,
 *     device- or host-resident IF buffers, status codes.  Used by the legacy
 *     shim below, by bench.py and by multi-GPU runners.
 *
 *  2. Legacy OSGPS register API (include/gnsscorr_osg.h): the exact symbols
 *     the reference's host side links against
 *       correlator_init / Sim_GP2021_int / REG_read / REG_write
 *     (reference osgnss_next_step/src/correlator/correlator.h:4-9), so the
 *     reference gp2021.c accessors and osgpsisr.c DLL/PLL link unchanged.
 *
 * All functions return 0 on success or a negative GNSSCORR_E* code.
 * Pointers named d_* are HIP device pointers; h_* are host pointers.
 * No torch types cross this boundary.
 */
#ifndef GNSSCORR_H
#define GNSSCORR_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNSSCORR_OK           0
#define GNSSCORR_EINVAL      -1   /* bad argument / shape                          */
#define GNSSCORR_ENOMEM      -2   /* device or host allocation failed              */
#define GNSSCORR_EDEVICE     -3   /* HIP runtime error (see gnsscorr_last_error)   */
#define GNSSCORR_ENODEV      -4   /* no HIP device visible                         */

/* Human-readable description of the last error on this thread. */
const char *gnsscorr_last_error(void);
/* Library version string. */
const char *gnsscorr_version(void);
/* Number of visible HIP devices (0 on a CPU-only host; never initialises
 * more than hipGetDeviceCount does). */
int gnsscorr_device_count(void);
/* LDS bytes one workgroup may allocate on a device: 160 KiB on gfx950 (the
 * per-CU attribute; the per-block one may report 64 KiB there), HIP's
 * per-block attribute elsewhere; 0 if it cannot be read.
 * Kernels that size their LDS at launch (per-channel IF staging) check it. */
int gnsscorr_device_lds_bytes(int device);
/* PCI bus id ("0000:xx:00.0") of a device, for run records. */
int gnsscorr_device_pci_bus_id(int device, char *buf, int len);
/* Path of the libamdhip64 whose hipMalloc this library calls, and
 * hipRuntimeGetVersion() of it (for run records: a host process may map a
 * second HIP runtime, e.g. PyTorch's). */
int gnsscorr_hip_runtime(char *path, int len, int *version);

/* ======================================================================
 * IF sample formats.  Every batched entry point that takes IF samples has an
 * `iq` argument (or gnsscorr_track_cfg.iq): a set of these flags.
 *   0                      int8 real samples, one byte each
 *   GNSSCORR_IF_IQ         int8 interleaved I,Q (two bytes per sample)
 *   | GNSSCORR_IF_PACKED2  2-bit codes, four elements per byte: element e of a
 *                          stream (I,Q,I,Q,... when complex) in bits
 *                          2*(e%4)..2*(e%4)+1 of byte e/4; code c is the level
 *                          2c-3, the GN3S LUT {-3,-1,1,3} of GPS_Source::Read_GN3S
 *                          (REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER/
 *                          objects/gps_source.cpp:692).  Results equal the int8
 *                          path on the unpacked levels; HBM and PCIe bytes are 1/4.
 * Strides and sample counts stay in samples; byte offsets of packed data are
 * element offsets / 4 (stream strides must make them whole 16-byte multiples
 * on the device).
 * ==================================================================== */
#define GNSSCORR_IF_IQ      1
#define GNSSCORR_IF_PACKED2 2
/* Host helper: pack n int8 levels in {-3,-1,1,3} into (n+3)/4 bytes of
 * GNSSCORR_IF_PACKED2 codes.  Returns GNSSCORR_EINVAL (and packs nothing) if a
 * value is not one of the four levels. */
int gnsscorr_pack2(const int8_t *h_in, int64_t n, uint8_t *h_out);

/* ======================================================================
 * Tracking correlator (GP2021 integer semantics)
 * Replaces: Sim_GP2021_int, osgnss_next_step/src/correlator/correlator.c:148-316
 * ==================================================================== */

#define GNSSCORR_OSG_ROW 2046      /* half-chips per C/A period */

typedef struct gnsscorr_track_ctx gnsscorr_track_ctx;

typedef struct {
  int    n_channels;     /* channels in this context (any number >= 1)           */
  int    iq;             /* GNSSCORR_IF_* flags: IQ = interleaved I,Q (use_iq_processing=1,
                            globals.h:56), else I only; | PACKED2 = 2-bit codes   */
  int    device;         /* HIP device ordinal                                    */
  int    max_nsamp;      /* largest nsamp per call (sizes the dump buffers)       */
  double samp_rate;      /* Hz, only used for tic_ref (correlator.c:124)          */
  double tic_period;     /* s; reference passes (int)0.1 == 0 (globals.h:52)     */
} gnsscorr_track_cfg;

/* What gp2021.c writes into REG_write for one channel (gp2021.c:75-130). */
typedef struct {
  int32_t  prn;          /* SATCNTL: 1..32, 0 = channel off                      */
  uint32_t carrier_incr; /* (REG_write[3]<<16)+REG_write[4]: per-sample carrier word */
  uint32_t code_incr;    /* (REG_write[5]<<16)+REG_write[6]; the NCO adds code_incr<<1 */
  uint32_t slew;         /* REG_write[(ch<<3)+0x84], 0..65535                    */
  int32_t  epoch_load;   /* -1: none; else REG_write[(ch<<3)+7] (16-bit)         */
  int32_t  stream;       /* IF stream index this channel correlates              */
} gnsscorr_nco_cmd;

/* struct gp2021_channel (correlator.c:36-47) + the ms/bit counters. */
typedef struct {
  uint32_t carrier_phase;
  uint32_t carrier_cycle;
  uint32_t code_phase;
  uint32_t half_chip;    /* uint16 semantics */
  int32_t  acc[6];       /* partial epoch: IL QL IP QP IE QE (REG_read order)    */
  int32_t  ms_counter;
  int32_t  bit_counter;
  int32_t  msbit_reg;    /* REG_read[(ch<<3)+7]                                  */
  int32_t  pad;
} gnsscorr_chan_state;

/* Per channel result of one call (what lands in REG_read). */
typedef struct {
  int32_t  n_dumps;      /* integrate-and-dump events in this call               */
  int32_t  dump[6];      /* LAST dump: IL QL IP QP IE QE (REG_read[(ch<<3)+0x84..]) */
  int32_t  msbit_reg;    /* REG_read[(ch<<3)+7] after the call                   */
  int32_t  tic;          /* 1 if the TIC latched this channel in this call       */
  int32_t  tic_regs[6];  /* REG_read[(ch<<3)+1..6] latched at the TIC            */
  int32_t  pad;
} gnsscorr_track_result;

int gnsscorr_track_create(gnsscorr_track_ctx **out, const gnsscorr_track_cfg *cfg);
int gnsscorr_track_destroy(gnsscorr_track_ctx *ctx);
/* Layout hint (kept for source compatibility, since 0.2.0 a validated no-op):
 * the kernel picks the load path per workgroup from the channels' streams --
 * receivers (channels sharing a stream) stage the stream once in LDS, channels
 * on distinct streams take the per-wave piece path -- so no hint is needed.
 * Returns GNSSCORR_EINVAL for a NULL context or a value other than 0 / 1. */
int gnsscorr_track_set_layout(gnsscorr_track_ctx *ctx, int one_stream_per_channel);
/* Max dumps one call can produce: floor(max_nsamp/2046)+2.  The optional
 * all-dumps buffer of gnsscorr_track() is n_channels * this * 6 int32. */
int gnsscorr_track_max_dumps(const gnsscorr_track_ctx *ctx);

/* One correlator call (one "interrupt") over nsamp samples for every channel.
 * h_if: host IF, n_streams streams of stream_stride samples each (bytes =
 * samples * (iq ? 2 : 1)); channel c reads stream cmds[c].stream.
 * NCO words take effect at the start of the call (reference semantics).
 * h_res: n_channels results; h_all_dumps: optional (may be NULL).
 * Returns whether the TIC fired through *tic_fired (may be NULL). */
int gnsscorr_track(gnsscorr_track_ctx *ctx, const int8_t *h_if, int64_t stream_stride,
                   int n_streams, int64_t nsamp, const gnsscorr_nco_cmd *h_cmds,
                   gnsscorr_track_result *h_res, int32_t *h_all_dumps, int *tic_fired);

/* Device-resident variant: IF, commands and results stay in HBM; the call is
 * asynchronous on the context stream (no host sync).  d_cmds / d_res /
 * d_all_dumps are device arrays sized as in gnsscorr_track().
 * tic_count: sample index of the TIC in this call or -1 (host computes it with
 * gnsscorr_track_next_tic()). */
int gnsscorr_track_dev(gnsscorr_track_ctx *ctx, const int8_t *d_if, int64_t stream_stride,
                       int64_t nsamp, const gnsscorr_nco_cmd *d_cmds,
                       gnsscorr_track_result *d_res, int32_t *d_all_dumps, int64_t tic_count);
/* Bytes of `samples` consecutive samples of one stream in the context's format. */
int64_t gnsscorr_track_if_bytes(const gnsscorr_track_ctx *ctx, int64_t samples);
/* Advances the context's TIC counter by nsamp (correlator.c:155-165) and
 * returns the TIC sample index for that call, or -1. */
int64_t gnsscorr_track_next_tic(gnsscorr_track_ctx *ctx, int64_t nsamp);

/* Open-loop replay: n_steps consecutive calls of nsamp samples; step k reads
 * IF at d_if + k*nsamp*(iq?2:1) of every stream and commands
 * d_cmds[k*n_channels ..]; results d_res[k*n_channels ..].  Asynchronous. */
int gnsscorr_track_replay_dev(gnsscorr_track_ctx *ctx, const int8_t *d_if, int64_t stream_stride,
                              int64_t nsamp, int n_steps, const gnsscorr_nco_cmd *d_cmds,
                              gnsscorr_track_result *d_res);

int gnsscorr_track_get_state(gnsscorr_track_ctx *ctx, gnsscorr_chan_state *h_state);
int gnsscorr_track_set_state(gnsscorr_track_ctx *ctx, const gnsscorr_chan_state *h_state);
int gnsscorr_track_sync(gnsscorr_track_ctx *ctx);
/* The HIP stream (hipStream_t) the context launches on. */
void *gnsscorr_track_stream(gnsscorr_track_ctx *ctx);

/* ======================================================================
 * OSG channel loops on the GPU, bit-exact with gpsisr
 * (osgnss_next_step/src/isr/osgpsisr.c:360-768): per dump, the acquisition /
 * n-of-m confirm / FLL-assisted-PLL + DLL pull-in / tracking state machine in
 * the reference's fixed-point arithmetic (rss, fix_atan2, sqrt_newton, long =
 * int64), writing the next call's NCO words, slew and epoch load straight into
 * the device command array.  With gnsscorr_track_dev this closes the loop on
 * the GPU: no host round trip per 512-us interrupt.
 * ==================================================================== */
typedef struct {          /* tracking_channel (OSG/include/structs.h:86-131), loop fields */
  int32_t state;          /* 0 off, 1 acquisition, 2 confirm, 3 pull-in, 4 tracking */
  int32_t n_freq, i_confirm, n_thresh, codes, del_freq;
  int32_t sign_pos, prev_sign_pos, sign_count, ms_count, ms_set;
  int32_t search_max_prn_delay, search_max_f;
  int32_t cn0, bit;       /* char in the reference                               */
  int32_t exited;         /* 1: a dump reached CHANNEL_OFF (the reference exit(0)s) */
  int16_t accum[6];       /* struct accum order: iP qP iL qL iE qE (short)       */
  int16_t prev_accum[6];
  int64_t early_mag, prompt_mag, late_mag;            /* accum_mean            */
  int64_t cross, dot, carr_error, old_carr_error, freq_error;
  int64_t carr_nco, old_carr_nco, carr_freq, carr_freq_basis;
  int64_t code_error, old_code_error, code_freq, code_freq_basis, code_nco, old_code_nco;
  int64_t ch_time, carrier_freq, carrier_cold_corr;
  uint64_t ms_sign;
} gnsscorr_osg_loop;      /* 264 bytes */

typedef struct {          /* receiver constants the loops read (globals.h, init code) */
  int64_t carrier_ref, code_ref, d_freq;   /* gps_carrier_ref, gps_code_ref, d_freq */
  int32_t fll_i1, fll_i2, fll_i3;          /* FLL_a_PLL_i1..3                   */
  int32_t dll_i1, dll_i2;                  /* DLL_i1, DLL_i2                    */
  int32_t acq_thresh;                      /* acq_thresh (globals.h:38)         */
  int32_t confirm_m, n_of_m_thresh;        /* CONFIRM_M, N_OF_M_THRESH           */
  int32_t carrier_shift, code_shift;       /* MAX_DIGIT - {CARRIER,CODE}_NCO bits */
  double  clock_mult;                      /* SYSTEM_CLOCK_MULTIPLIER (double)  */
} gnsscorr_osg_loop_cfg;

/* Constants as the reference computes them at start-up: correlator_init
 * (correlator.c:110-121) and osgnss_next_step.c:391-399 (calc_* / convert_*,
 * osgpsisr.c:213-330).  Defaults of globals.h: fs 16e6, IF 2.42e6, clock x5,
 * NCO bits 30/29, bin 1000 Hz, Bnp 25, Bnf 1400, Bnd 2, 1 ms, acq_thresh 1800. */
void gnsscorr_osg_loop_cfg_init(gnsscorr_osg_loop_cfg *cfg, double samp_rate, double gps_if,
                                double clock_mult, int carrier_nco_bits, int code_nco_bits,
                                double bin_width, long bnp, long bnf, long bnd, long fll_t_ms,
                                long dll_t_ms, int acq_thresh);
/* The start state of osgnss_next_step.c:73-84 (reset_all_correlator_channles):
 * acquisition, n_freq 0, del_freq 1, 2045 half-chip delays, +-5 bins; cmds get
 * the PRN, the reference carrier/code words, no slew, no epoch load. */
void gnsscorr_osg_loop_reset(const gnsscorr_osg_loop_cfg *cfg, int n_ch, const int32_t *prns,
                             gnsscorr_osg_loop *loops, gnsscorr_nco_cmd *cmds);
/* One interrupt's channel processing after a gnsscorr_track_dev call that used
 * d_cmds and wrote d_res: register bookkeeping of the call (epoch load
 * consumed, slew cleared by a dump), then gpsisr for every channel that dumped.
 * Updates d_loops and d_cmds in place for the next call.  Asynchronous on the
 * tracking context's stream. */
int gnsscorr_osg_isr_dev(gnsscorr_track_ctx *ctx, const gnsscorr_osg_loop_cfg *cfg, int n_ch,
                         gnsscorr_osg_loop *d_loops, gnsscorr_nco_cmd *d_cmds,
                         const gnsscorr_track_result *d_res);
/* n_calls closed-loop interrupts: for k in 0..n_calls-1, gnsscorr_track_dev on
 * IF d_if + k*nsamp samples (every stream), then gnsscorr_osg_isr_dev.  The
 * per-call results (n_calls * n_ch) and loop states (optional, may be NULL)
 * are recorded for inspection.  Asynchronous. */
int gnsscorr_osg_closed_loop_dev(gnsscorr_track_ctx *ctx, const gnsscorr_osg_loop_cfg *cfg,
                                 const int8_t *d_if, int64_t stream_stride, int64_t nsamp,
                                 int n_calls, int n_ch, gnsscorr_osg_loop *d_loops,
                                 gnsscorr_nco_cmd *d_cmds, gnsscorr_track_result *d_res_hist,
                                 gnsscorr_osg_loop *d_loop_hist);

/* ======================================================================
 * Parallel code-phase acquisition (SoftGNSS acquisition.sci semantics)
 * Replaces: GPS  POSTPROCESSING_SCILAB_RECEIVERS/GPS/L1/acquisition.sci:46-192
 *           GLO  POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/acquisition.sci:46-198
 * ==================================================================== */

typedef struct gnsscorr_acq_ctx gnsscorr_acq_ctx;

/* Arithmetic of the acquisition kernels (gnsscorr_acq_cfg.precision).
 * F64 is the reference's own precision (Scilab evaluates acquisition.sci in
 * doubles): wipe-off, transforms, products, powers and comparisons in fp64;
 * n_samples 16368 (16.368 Msps) or 16000 (16 Msps, initSettings.sci:69).
 * F32 is the faster single-precision path, n_samples 16368 only; its rows
 * agree with fp64 to ~1e-5 of the row maximum. */
#define GNSSCORR_ACQ_F64 0
#define GNSSCORR_ACQ_F32 1

typedef struct {
  double samp_rate;       /* settings.samplingFreq                                 */
  int    n_samples;       /* samplesPerCode = round(fs/(codeFreq/codeLength))       */
  int    device;
  int    max_freqs;       /* capacity of the carrier-frequency table               */
  int    max_blocks;      /* capacity of 1-ms IF blocks per search                 */
  int    max_codes;       /* capacity of the code table                            */
  int    precision;       /* GNSSCORR_ACQ_F64 (default, 0) or GNSSCORR_ACQ_F32      */
} gnsscorr_acq_cfg;

/* Statistics of one correlation row (code x carrier frequency [x block]). */
typedef struct {
  double  peak;           /* max |ifft|^2 of the row                               */
  double  second;         /* max outside the open +-spc window around argmax       */
  int32_t argmax;         /* 0-based sample index of the first maximum             */
  int32_t block;          /* which block the stats come from (best-of-blocks mode) */
} gnsscorr_acq_row;

/* Per search group (one PRN / FCH), acquisition.sci:141-186. */
typedef struct {
  double  peak;           /* peakSize                                              */
  double  second;         /* secondPeakSize                                        */
  double  metric;         /* peakSize / secondPeakSize                             */
  int32_t bin;            /* 0-based frequencyBinIndex-1                           */
  int32_t code_phase;     /* 1-based codePhase (as acquisition.sci returns it)     */
  int32_t pad;            /* 1: an exact tie put the first column in another row   */
  int32_t pad2;
  double  carr_freq;      /* carrier frequency of the winning bin [Hz]             */
} gnsscorr_acq_result;

#define GNSSCORR_ACQ_BEST_OF_BLOCKS 0  /* SoftGNSS: keep the block with larger max */
#define GNSSCORR_ACQ_NONCOHERENT    1  /* sum |.|^2 over blocks before the search  */

int gnsscorr_acq_create(gnsscorr_acq_ctx **out, const gnsscorr_acq_cfg *cfg);
int gnsscorr_acq_destroy(gnsscorr_acq_ctx *ctx);
/* Upload n_codes sampled code replicas (n_samples int8 values of +-1 each,
 * e.g. makeCaTable.sci / makeStTable.sci rows); their spectra are computed on
 * the device and kept resident. */
int gnsscorr_acq_set_codes(gnsscorr_acq_ctx *ctx, int n_codes, const int8_t *h_codes);
/* The code replicas generated on the device from code ids, then their spectra:
 * what acquisition.sci:91-95 does at the start of every search
 * (caCodesTable = makeCaTable(settings); conj(fft(caCodesTable(PRN,:)))).  Id p
 * in 1..32 is GPS C/A PRN p (generateCAcode.sci, sampled at 1.023 MHz chips by
 * makeCaTable.sci:64-72); GNSSCORR_CODE_GLO_ST is the GLONASS ST code
 * (generateSTcode.sci, 0.511 MHz chips, makeStTable.sci:60-67).  Same replicas,
 * bit for bit, as gnsscorr_ca_code / gnsscorr_st_code + gnsscorr_sample_code
 * uploaded with gnsscorr_acq_set_codes.  Asynchronous on the context stream, no
 * allocation after the first call (the chip table, 33 x 1023 B, is built then). */
#define GNSSCORR_CODE_GLO_ST 0
int gnsscorr_acq_set_prn_codes(gnsscorr_acq_ctx *ctx, int n_codes, const int32_t *h_code_ids);

/* Search.  IF: n_blocks consecutive blocks of n_samples samples, format
 * `iq` (GNSSCORR_IF_* flags: interleaved I,Q or real, int8 or 2-bit packed).  freqs: n_freqs carrier
 * frequencies [Hz] (wipe-off exp(i*2*pi*f*t), t = n/fs).  Groups: n_groups
 * searches, each of n_bins rows: group g uses code group_code[g] and
 * frequency index group_freq[g*n_bins + b] for bin b.
 * spc = samplesPerCodeChip (exclusion half-width for the second peak).
 * Outputs: h_rows (n_groups*n_bins, may be NULL), h_res (n_groups). */
int gnsscorr_acq_search(gnsscorr_acq_ctx *ctx, const int8_t *h_if, int iq, int n_blocks,
                        int mode, int n_freqs, const double *h_freqs, int n_groups,
                        int n_bins, const int32_t *h_group_code, const int32_t *h_group_freq,
                        int spc, gnsscorr_acq_row *h_rows, gnsscorr_acq_result *h_res);

/* Device-resident variant (asynchronous; d_rows / d_res device arrays).  The
 * group tables and frequencies are device arrays too. */
int gnsscorr_acq_search_dev(gnsscorr_acq_ctx *ctx, const int8_t *d_if, int iq, int n_blocks,
                            int mode, int n_freqs, const double *d_freqs, int n_groups,
                            int n_bins, const int32_t *d_group_code, const int32_t *d_group_freq,
                            int spc, gnsscorr_acq_row *d_rows, gnsscorr_acq_result *d_res);

/* The two stages of gnsscorr_acq_search_dev, for re-correlating resident
 * spectra with another code set or timing the stages separately:
 *  spectra:   wipe-off + FFT of every (freq, block), kept in the context
 *  correlate: conj-multiply + IFFT + |.|^2 + peak search of every group row;
 *             with d_rows the rows are combined over blocks (and with d_res
 *             the per-group selection runs too); with both NULL the per-block
 *             statistics stay in the context for gnsscorr_acq_select_dev(). */
int gnsscorr_acq_spectra_dev(gnsscorr_acq_ctx *ctx, const int8_t *d_if, int iq, int n_blocks,
                             int n_freqs, const double *d_freqs);
int gnsscorr_acq_correlate_dev(gnsscorr_acq_ctx *ctx, int n_blocks, int mode,
                               const double *d_freqs, int n_groups, int n_bins,
                               const int32_t *d_group_code, const int32_t *d_group_freq, int spc,
                               gnsscorr_acq_row *d_rows, gnsscorr_acq_result *d_res);

/* Block combine (acquisition.sci:126-132) + per-group selection (:141-186)
 * over the statistics of the last correlate call; writes d_rows (and d_res
 * when not NULL). */
int gnsscorr_acq_select_dev(gnsscorr_acq_ctx *ctx, int n_groups, int n_bins, const double *d_freqs,
                            const int32_t *d_group_freq, gnsscorr_acq_row *d_rows,
                            gnsscorr_acq_result *d_res);

/* Coherent integration of settings.acqCohIntegration code periods per block
 * (GLONASS acquisition.sci:52-72, default 5): every block of the following
 * searches is coh_ms x n_samples samples, wiped off with one continuous phase
 * ramp and correlated against the code repeated coh_ms times; rows hold the
 * first code period of |ifft|^2 as acquisition.sci keeps them.  Needs
 * n_blocks * coh_ms <= max_blocks.  Default 1. */
int gnsscorr_acq_set_coherent(gnsscorr_acq_ctx *ctx, int coh_ms);
/* Several records per search (fp64 precision; n_samples 16368 or 16000, or a
 * generic n_samples with no prime factor above 31): the following searches read
 * n_records IF records laid end to end, record r at
 * sample r * n_blocks * coh_ms * n_samples (IQ pairs counted as one sample),
 * and search every record with the same frequencies and groups -- as
 * n_records separate acquisition.sci calls, in one correlation launch (the
 * generic engine: one chunk loop over every record's units).
 * Outputs are record-major: res[r * n_groups + g], rows[(r * n_groups + g) *
 * n_bins + b]; d_rows / d_res (and h_rows / h_res) hold n_records times as
 * many entries.  Needs n_records * n_blocks * coh_ms <= max_blocks.
 * Default 1.  (acquisition.sci:46-192 per record; no reference counterpart
 * for the batching itself.) */
int gnsscorr_acq_set_records(gnsscorr_acq_ctx *ctx, int n_records);
/* Per-group records: with d_group_rec (device, one int32 per group, values in
 * [0, records)) a correlate call searches group g on record d_group_rec[g] only,
 * instead of every group on every record; results are per group.  Lets one launch
 * hold groups of different IF streams (the GPS and GLONASS records of a full-sky
 * search).  NULL turns it off.  fp64 compiled plans only; the array must stay
 * valid while correlate calls use it.  A value outside [0, records) is clamped
 * into that range; gnsscorr_acq_set_records with another count turns the table
 * off (set it again after).  (No reference counterpart: batching.) */
int gnsscorr_acq_set_group_records(gnsscorr_acq_ctx *ctx, const int32_t *d_group_rec);
/* Debug/parity: full |ifft|^2 power row for (code, freq, block): n_samples doubles. */
int gnsscorr_acq_power_row(gnsscorr_acq_ctx *ctx, const int8_t *h_if, int iq, int n_blocks,
                           int block, double freq, int code, double *h_power);
int gnsscorr_acq_sync(gnsscorr_acq_ctx *ctx);
void *gnsscorr_acq_stream(gnsscorr_acq_ctx *ctx);

/* ======================================================================
 * SoftGNSS float tracking ("sgt"): the Scilab receivers' per-channel loop
 *   GLONASS POSTPROCESSING_SCILAB_RECEIVERS/GLONASS/L1/tracking.sci:150-400
 *   GPS     POSTPROCESSING_SCILAB_RECEIVERS/GPS/L1/tracking.sci:124-360
 * One epoch = one code period: blksize = ceil((L - remCode)/step) samples,
 * E/P/L replica indices ceil(remCode -/+ spc + k*step) (fp64, bit-exact),
 * carrier exp(i*(2*pi*f*t + remCarr)) (fp64), six fp64 sums
 * I = sum(code*imag(carr*raw)), Q = sum(code*real(carr*raw)), then (closed
 * loop) the FLL-assisted PLL and the DLL of tracking.sci:329-375 on the GPU.
 * The IF record(s) stay resident in HBM; each channel reads from its own
 * position (the reference's per-channel mseek, tracking.sci:163-168).
 * ==================================================================== */
typedef struct gnsscorr_sgt_ctx gnsscorr_sgt_ctx;

typedef struct {          /* initSettings.sci fields used by tracking.sci     */
  int32_t system;         /* 0 = GPS L1 C/A (C/A code per PRN), 1 = GLONASS L1OF (ST) */
  int32_t file_type;      /* settings.fileType: 1 = int8 real, 2 = int8 interleaved I,Q */
  int32_t switch_iq;      /* settings.switchIQ (GLONASS only, tracking.sci:263-267) */
  int32_t code_length;    /* settings.codeLength: 1023 / 511                   */
  int32_t device;
  int32_t max_channels;
  double  samp_rate;      /* settings.samplingFreq                             */
  double  code_freq_basis;/* settings.codeFreqBasis                            */
  double  if_freq;        /* settings.IF                                       */
  double  l1_if_step;     /* settings.L1_IF_step (GLONASS)                      */
  double  glonass_zero_channel; /* settings.GLONASS_zero_channel               */
  double  dll_spacing;    /* settings.dllCorrelatorSpacing [chips]             */
  double  dll_noise_bw, dll_damping;   /* calcLoopCoef(dllNoiseBandwidth, dllDampingRatio, 1) */
  double  pll_noise_bw, fll_noise_bw;  /* calcFLLPLLLoopCoef(pll, fll, PDIcarr=0.001) */
  /* tracking.sci variants; 0 = the current file for both.  The reference's
   * recorded runs (GLONASS/L1,L2/trackingResults.dat) used 1 and 1. */
  int32_t code_nco_variant;   /* 0: codeFreq with carrier aiding (:367-370, GPS :1540 form);
                                 1: codeFreq = codeFreqBasis - codeNco (:366)          */
  int32_t abs_sample_variant; /* 0: currentSample - remCodePhase*(fs/1000)/L (:384);
                                 1: mtell(fid)/dataAdaptCoeff, whole samples (:379)    */
} gnsscorr_sgt_cfg;

typedef struct {          /* one tracking channel (tracking.sci:159-201 + loop state) */
  int32_t code_id;        /* GPS PRN 1..32, or GLONASS FCH -7..6                */
  int32_t stream;         /* which IF record (stride given per call)           */
  int32_t status;         /* 0 tracking, 1 out of data (tracking.sci:273-277)  */
  int32_t n_epochs;       /* epochs processed so far                           */
  int64_t pos;            /* next sample (complex or real) of the record       */
  int64_t pad;
  double  rem_code, rem_carr, code_freq, carr_freq, carr_freq_basis;
  double  old_code_nco, old_code_error, old_carr_nco, old_carr_error, i1, q1;
  double  pad2;
} gnsscorr_sgt_chan;      /* 128 bytes */

typedef struct {          /* trackResults(ch).* for one epoch (tracking.sci:387-398) */
  double  i_e, i_p, i_l, q_e, q_p, q_l;
  double  carr_freq, code_freq, absolute_sample;
  double  dll_discr, dll_discr_filt, pll_discr, pll_discr_filt;
  int32_t blksize;        /* samples of the epoch; on a stop record the blksize that did
                             not fit, or -1 if it is not a representable count (NaN, or
                             2^31 or more: a corrupted state, which also stops) */
  int32_t status;         /* 0 ok; 1 = this epoch was not processed (out of data) */
} gnsscorr_sgt_epoch;     /* 112 bytes */

/* Loop coefficients exactly as calcLoopCoef.sci:39-43 / calcFLLPLLLoopCoef.sci:36-38. */
void gnsscorr_sgt_loop_coefs(const gnsscorr_sgt_cfg *cfg, double *tau1code, double *tau2code,
                             double *k1, double *k2, double *k3);
/* Channel initialisation from an acquisition result (tracking.sci:159-201):
 * pos = skip_samples + code_phase_1b - 1, codeFreq = basis, carrFreq = acquiredFreq. */
int gnsscorr_sgt_init_chan(const gnsscorr_sgt_cfg *cfg, int code_id, int stream,
                           int64_t skip_samples, int64_t code_phase_1b, double acquired_freq,
                           gnsscorr_sgt_chan *out);
int gnsscorr_sgt_create(gnsscorr_sgt_ctx **out, const gnsscorr_sgt_cfg *cfg);
int gnsscorr_sgt_destroy(gnsscorr_sgt_ctx *ctx);
/* Run n_epochs epochs of n_ch channels (state in d_chan, updated in place).
 * d_if: the records, stream s at d_if + s*stream_stride bytes, each
 * n_samples samples long.  closed_loop=1: the loop filters of tracking.sci
 * update codeFreq/carrFreq after every epoch; 0: correlator only, frequencies
 * held (a host-side loop updates them between calls).  d_epochs[ch*n_epochs+e]
 * receives the per-epoch record.  Asynchronous on the context's stream. */
int gnsscorr_sgt_track_dev(gnsscorr_sgt_ctx *ctx, const int8_t *d_if, int64_t stream_stride,
                           int64_t n_samples, int n_ch, gnsscorr_sgt_chan *d_chan,
                           int n_epochs, int closed_loop, gnsscorr_sgt_epoch *d_epochs);
/* Same with host channel state / results (synchronous). */
int gnsscorr_sgt_track(gnsscorr_sgt_ctx *ctx, const int8_t *d_if, int64_t stream_stride,
                       int64_t n_samples, int n_ch, gnsscorr_sgt_chan *h_chan, int n_epochs,
                       int closed_loop, gnsscorr_sgt_epoch *h_epochs);
/* The loop half alone (tracking.sci:248-252, 301-313, 329-398): n_epochs
 * epochs of n_ch channels driven by given correlator sums instead of a record,
 * sums[(ch*n_epochs + e)*6 + j], j = I_E, I_P, I_L, Q_E, Q_P, Q_L.  Runs the
 * same device code as the closed-loop tracker (blksize / remCodePhase chain,
 * discriminators, filters, NCO frequencies, absoluteSample).  For a host that
 * correlates elsewhere, and to replay a recorded trackResults.  _dev:
 * device buffers, asynchronous on the context's stream; without: host
 * buffers, synchronous. */
int gnsscorr_sgt_replay_dev(gnsscorr_sgt_ctx *ctx, int n_ch, gnsscorr_sgt_chan *d_chan,
                            int n_epochs, const double *d_sums, gnsscorr_sgt_epoch *d_epochs);
int gnsscorr_sgt_replay(gnsscorr_sgt_ctx *ctx, int n_ch, gnsscorr_sgt_chan *h_chan,
                        int n_epochs, const double *h_sums, gnsscorr_sgt_epoch *h_epochs);
int gnsscorr_sgt_sync(gnsscorr_sgt_ctx *ctx);
void *gnsscorr_sgt_stream(gnsscorr_sgt_ctx *ctx);

/* ======================================================================
 * GPS-SDR integer strong acquisition ("sdr"), bit-exact with the real-time
 * receiver's int16 path (REALTIME_RECEIVERS/GPS/GPS_SDR_REAL_TIME_GPS_RECEIVER):
 *   Acquisition::doPrepIF    objects/acquisition.cpp:191-236 (1 ms buffer)
 *   Acquisition::doAcqStrong objects/acquisition.cpp:244-301
 * Input: CPX buffers of 2048 int16 (I, Q) pairs = 1 ms at 2.048 Msps
 * (defines.h:150-151), IF fif (signaldef.h:34: 38.4 kHz).  Per sv (0-based
 * index into PRN_Codes, MAX_SV = 32): 4 sub-bins (0/250/500/750 Hz) x 1 kHz
 * circular spectrum shifts lcv in [doppmin/1000, doppmax/1000), int16 FFTs
 * with the reference's Q14 twiddles, rank scaling and wrap points.
 * ==================================================================== */
typedef struct gnsscorr_sdr_acq_ctx gnsscorr_sdr_acq_ctx;

typedef struct {
  double  fif;            /* IF [Hz]: the wipe-offs are sine_gen(-fif - 250*j) */
  int32_t device;
  int32_t saturate;       /* 1: sse_cmulsc packssdw saturation (production);
                             0: x86_cmulsc int16 wrap (the -DNO_SIMD build)   */
} gnsscorr_sdr_acq_cfg;

typedef struct {          /* Acq_Command_S result fields (structs.h:130-164) */
  int32_t  sv;
  int32_t  code_phase;    /* 2048 - argmax                                   */
  int32_t  doppler;       /* lcv*1000 + lcv2*250                             */
  uint32_t magnitude;     /* I^2 + Q^2 of the peak (int32 arithmetic)        */
  int32_t  success;       /* magnitude > THRESH_STRONG (= 0, config.h:72)    */
  int32_t  row;           /* winning row (lcv - doppmin/1000)*4 + lcv2       */
} gnsscorr_sdr_acq_result;

/* PRN_Codes (accessories/prn_codes.h, generated by gen_fft_codes.m): 51 PRNs x
 * 2048 (re, im) int16 = conj(FFT(resampled code)) scaled to 9 bits. */
int gnsscorr_sdr_prn_codes(int16_t *h_out);
/* sine_gen (accessories/misc.cpp:95-115): n (i, q) int16 pairs. */
void gnsscorr_sdr_sine_gen(int16_t *h_out, double f, double fs, int n);
int gnsscorr_sdr_acq_create(gnsscorr_sdr_acq_ctx **out, const gnsscorr_sdr_acq_cfg *cfg);
int gnsscorr_sdr_acq_destroy(gnsscorr_sdr_acq_ctx *ctx);
/* n_rec buffers (each 2048 CPX) x n_sv svs -> h_res[rec*n_sv + s].  Requires
 * -100 <= doppmin/1000 < doppmax/1000 <= 101 (the reference's +-100-bin row
 * padding, acquisition.cpp:229-233) and 0 <= sv < 32. */
int gnsscorr_sdr_acq_strong(gnsscorr_sdr_acq_ctx *ctx, const int16_t *h_buff, int n_rec, int n_sv,
                            const int32_t *h_svs, int doppmin, int doppmax,
                            gnsscorr_sdr_acq_result *h_res);
int gnsscorr_sdr_acq_strong_dev(gnsscorr_sdr_acq_ctx *ctx, const int16_t *d_buff, int n_rec,
                                int n_sv, const int32_t *d_svs, int doppmin, int doppmax,
                                gnsscorr_sdr_acq_result *d_res);
/* ---- medium / weak acquisition (SDR/objects/acquisition.cpp:191-236,
 * 309-570; replaces Acquisition::Acquire's doPrepIF + doAcqMedium / doAcqWeak).
 * The context keeps, per record, the reference object's baseband_rows member:
 * 1240 prepared 1-ms spectra that persist between calls.  A prep of type t
 * writes rows 0 .. 4*ms-1 (ms = 1 / 10 / 310) and leaves the rest as they
 * were (zero at creation).  doAcqMedium reads rows lcv2*20 + 0..9 after a
 * 10-ms prep, so for lcv2 >= 2 it sees rows an earlier weak prep left; this
 * is reproduced.  Results: code_phase = argmax % 2048 (no 2048 - x here),
 * doppler = lcv*1000 + lcv2*250 + (argmax / 2048)*25, row = (lcv - lmin)*4 +
 * lcv2 (medium) or ((lcv - lmin)*4 + lcv2)*2 + k (weak, k = even/odd 10 ms). */
#define GNSSCORR_SDR_ACQ_STRONG 0  /* ACQ_TYPE_STRONG: 1 ms                     */
#define GNSSCORR_SDR_ACQ_MEDIUM 1  /* ACQ_TYPE_MEDIUM: 10 ms coherent + DFT     */
#define GNSSCORR_SDR_ACQ_WEAK   2  /* ACQ_TYPE_WEAK: 15 x (10 ms + DFT) non-coh */
/* d_buff: n_rec records of ms x 2048 CPX each (ms = 1 / 10 / 310 by type). */
int gnsscorr_sdr_acq_prep_dev(gnsscorr_sdr_acq_ctx *ctx, int type, const int16_t *d_buff,
                              int n_rec);
/* type MEDIUM: -100 <= doppmin/1000 <= doppmax/1000 <= 100 (lcv inclusive);
 * type WEAK:   -100 <= doppmin/1000 <  doppmax/1000 <= 101 (lcv exclusive). */
int gnsscorr_sdr_acq_search_dev(gnsscorr_sdr_acq_ctx *ctx, int type, int n_rec, int n_sv,
                                const int32_t *d_svs, int doppmin, int doppmax,
                                gnsscorr_sdr_acq_result *d_res);
/* Acquisition::Acquire for one request type over host buffers: prep + search. */
int gnsscorr_sdr_acq_acquire(gnsscorr_sdr_acq_ctx *ctx, int type, const int16_t *h_buff,
                             int n_rec, int n_sv, const int32_t *h_svs, int doppmin, int doppmax,
                             gnsscorr_sdr_acq_result *h_res);
int gnsscorr_sdr_acq_sync(gnsscorr_sdr_acq_ctx *ctx);
void *gnsscorr_sdr_acq_stream(gnsscorr_sdr_acq_ctx *ctx);

/* ======================================================================
 * GPS-SDR tracking correlator ("sdr corr"), bit-exact with the real-time
 * receiver's Correlator class (objects/correlator.cpp):
 *   Correlator::Accum       :425-448  wipe-off (cmulsc >>14) + E/P/L prn_accum_new
 *                            -> batched on the GPU (gnsscorr_sdr_accum_dev)
 *   Correlator::Correlate   :160-237  the per-packet rollover / dump schedule
 *   UpdateState / DumpAccum :369-525  fp64 NCO state, correlation rotation
 *   InitCorrelator          :610-676
 * Pre-sampled tables as in the constructor/SamplePRN (:63-98, :562-590):
 * 3001 carrier rows (-IF - 10 Hz*k, |k| <= 1500) x 4096 CPX and 32 SVs x 101
 * fractional-chip code rows x 4096 samples, resident in HBM.  The channel
 * DLL/PLL (Channel::Accum) stays host code: a callback per dump.
 * ==================================================================== */
typedef struct gnsscorr_sdr_corr_ctx gnsscorr_sdr_corr_ctx;

typedef struct {
  int32_t device;
  int32_t saturate;        /* 1: sse_cmulsc saturation; 0: x86_cmulsc wrap */
} gnsscorr_sdr_corr_cfg;

typedef struct {           /* Correlator_State_S (sdr_structs.h:141-168); the row
                              pointers pcode[3]/psine become (bin, offset) pairs */
  double   code_phase, carrier_phase, carrier_phase_prev, code_phase_mod, carrier_phase_mod;
  double   code_nco, carrier_nco;
  uint32_t chan, sv, navigate, active, count, scount;
  uint32_t epoch_1ms, epoch_20ms, z_count, rollover;
  uint32_t cbin[3], sbin;
  int32_t  coff[3], soff;
} gnsscorr_sdr_chan;       /* 128 bytes */

typedef struct { int32_t i[3], q[3]; } gnsscorr_sdr_corr;        /* Correlation_S: E, P, L */

typedef struct {           /* NCO_Command_S (sdr_structs.h:112-125) */
  double   carrier_nco, code_nco;
  uint32_t kill, reset_1ms, reset_20ms, set_z_count, z_count, length, navigate, pad;
} gnsscorr_sdr_feedback;

/* Channel::Accum stand-in: called at every dump with the rotated correlations;
 * fills the feedback (the struct is zeroed before the call). */
typedef void (*gnsscorr_sdr_dump_fn)(void *user, int ch, const gnsscorr_sdr_chan *s,
                                     const gnsscorr_sdr_corr *c, gnsscorr_sdr_feedback *f);

typedef struct {           /* one Correlator::Accum call */
  int32_t packet, data_off, samps;  /* samples [data_off, data_off+samps) of packet   */
  int32_t sv, sbin, soff;           /* carrier row sbin from offset soff              */
  int32_t cbin[3], coff[3];         /* E, P, L code rows of sv from offsets coff[]    */
} gnsscorr_sdr_accum_job;  /* 48 bytes */

int gnsscorr_sdr_corr_create(gnsscorr_sdr_corr_ctx **out, const gnsscorr_sdr_corr_cfg *cfg);
int gnsscorr_sdr_corr_destroy(gnsscorr_sdr_corr_ctx *ctx);
/* InitCorrelator from an acquisition result (sv 0-based, code_phase in samples,
 * doppler Hz) and the packets elapsed since the acquisition's buffer. */
int gnsscorr_sdr_init_chan(gnsscorr_sdr_chan *s, int sv, int acq_code_phase, int acq_doppler,
                           double packets_since_acq);
/* Batched Accum: d_packets = n x 2048 CPX on the device; d_out[j] = the E,P,L
 * sums of job j (int32, wrapping).  Asynchronous on the context stream. */
int gnsscorr_sdr_accum_dev(gnsscorr_sdr_corr_ctx *ctx, const int16_t *d_packets, int n_jobs,
                           const gnsscorr_sdr_accum_job *d_jobs, gnsscorr_sdr_corr *d_out);
/* Correlator::Correlate for one packet per receiver: h_packets = n_packets x
 * 2048 CPX (host), channel c reads packet h_rx[c] (NULL: all packet 0).
 * states/corr: n_ch entries updated in place; cb runs on the calling thread at
 * every dump, in channel order within each of the (at most 3) segment phases. */
int gnsscorr_sdr_correlate(gnsscorr_sdr_corr_ctx *ctx, const int16_t *h_packets, int n_packets,
                           int n_ch, const int32_t *h_rx, gnsscorr_sdr_chan *states,
                           gnsscorr_sdr_corr *corr, gnsscorr_sdr_dump_fn cb, void *user);
int gnsscorr_sdr_corr_sync(gnsscorr_sdr_corr_ctx *ctx);
void *gnsscorr_sdr_corr_stream(gnsscorr_sdr_corr_ctx *ctx);
/* Device the context was created on (-1 for NULL). */
int gnsscorr_sdr_corr_device(const gnsscorr_sdr_corr_ctx *ctx);

/* ======================================================================
 * GPS-SDR channel: Channel::Accum
 * (objects/channel.cpp:182-279) batched over channels on the GPU, one thread
 * per channel running its 1-ms calls in order:
 *   integrate / 20-ms running sums / bit-edge histogram   :185-213
 *   DumpAccum: powers, P_avg, FrequencyLock (512-point int16 FFT of the
 *              squared prompt), PLL (3rd order), DLL, Error/Kill  :282-500, 945-993
 *   EstCN0 :322-355, BitLock :524-611, BitStuff :615-651,
 *   ProcessDataBit / FrameSync / ParityCheck / ValidFrameFormat :655-904,
 *   Epoch :502-518, NCO_Command_S feedback :227-278.
 * Integer state, bit decisions, frame sync, parity and subframes are exact;
 * the float / double loop state follows the reference's float/double
 * expression types with FMA contraction off (atan / log10 may differ from
 * glibc in the last bit).  Valid subframes (ProcessDataBit's pipe write to
 * the ephemeris task, :687) come out as gnsscorr_sdr_subframe events.
 * ==================================================================== */
typedef struct {           /* the Channel object's state (objects/channel.h:53-132) */
  double   carrier_nco, code_nco;
  int32_t  len, count, state, sv, chan;     /* state: 0 EMPTY .. 3 NORMAL          */
  int32_t  I[3], Q[3], P[3], I_prev, Q_prev;
  float    I_avg, Q_var, P_avg, cn0;
  int32_t  bit_lock, bit_lock_pend, bit_lock_ticks, I_sum20, Q_sum20;
  int32_t  I_buff[20], Q_buff[20], P_buff[20];
  int32_t  epoch_20ms, epoch_1ms, best_epoch;
  int32_t  valid_frame[5], navigate, z_lock, converged, frame_z, z_count, z_count_pend;
  uint32_t word_buff[12];
  int32_t  frame_lock, frame_lock_pend, bit_number, subframe;
  int32_t  freq_lock, freq_lock_ticks;
  float    pll[17];        /* Phase_lock_loop: PLLBW FLLBW a3 b3 w0p w0p2 w0p3 a2 w0f w0f2
                              gain w x z pll_lock fll_lock t (fll_lock: see DESIGN.md) */
  float    dll[7];         /* Delay_lock_loop: DLLBW x z a w0 w02 t                    */
  uint32_t fft_buff[512];  /* CPX fft_buff[FREQ_LOCK_POINTS]                          */
} gnsscorr_sdr_channel;    /* 2632 bytes */

typedef struct {           /* Channel_2_Ephemeris_S (structs.h:60-66) + where / when */
  int32_t  sv, subframe;
  uint32_t word_buff[12];
  int32_t  chan, ms;       /* channel index and 1-ms call index within the launch   */
} gnsscorr_sdr_subframe;

/* Channel::Clear + Channel::Start (channel.cpp:71-170): corr_len 1 or 20. */
int gnsscorr_sdr_channel_start(gnsscorr_sdr_channel *ch, int chan, int sv, int acq_doppler,
                               int corr_len);
/* n_ms calls of Channel::Accum for each of n_ch channels: d_corr[m*n_ch + c]
 * is channel c's Correlation_S of call m (E, P, L); d_fb[m*n_ch + c] gets the
 * NCO_Command_S it fills (d_fb NULL: only the last call's, in d_fb_last).
 * Valid subframes are appended to d_events (up to max_events; *d_n_events
 * counts them all; slots are taken in arrival order, so sort by (call,
 * channel)).  On overflow (*d_n_events > max_events) WHICH subframes were
 * kept is arbitrary: size max_events from n_ch * n_ms / 6000 + n_ch (one
 * subframe per 6 s per channel) or retry larger.  Async on the context stream. */
int gnsscorr_sdr_channel_accum_dev(gnsscorr_sdr_corr_ctx *ctx, int n_ch, int n_ms,
                                   const gnsscorr_sdr_corr *d_corr, gnsscorr_sdr_channel *d_ch,
                                   gnsscorr_sdr_feedback *d_fb, gnsscorr_sdr_feedback *d_fb_last,
                                   gnsscorr_sdr_subframe *d_events, int max_events,
                                   int32_t *d_n_events);

/* Device-resident closed loop: Correlator::Correlate
 * (correlator.cpp:160-237) over n_packets consecutive packets, with
 * UpdateState, DumpAccum and Channel::Accum + ProcessFeedback (:452-555) at
 * every dump, without a host round trip -- channel c's Channel object d_ch[c]
 * steers correlator d_states[c].  One workgroup per channel.
 * d_packets: n_packets x n_rx x 2048 CPX (packet-major); channel c reads
 * receiver d_rx[c] (NULL: 0).  d_states / d_corr / d_ch: n_ch entries,
 * updated in place.  d_fb_last[c] (optional): the last dump's feedback.
 * d_log (optional): log_per_ch records per channel (channel-major), the first
 * log_per_ch dumps; d_n_log[c] (optional) counts all of channel c's dumps.
 * d_status[c]: 0; 1 + p when the state left the tables at packet p (the
 * channel stops there -- the host path returns GNSSCORR_EINVAL instead);
 * -1 for a receiver index outside 0..n_rx-1.  Subframe events as in
 * gnsscorr_sdr_channel_accum_dev with ms = the packet index.  Bit-identical
 * to gnsscorr_sdr_correlate packet by packet with gnsscorr_sdr_channel_accum_dev
 * as the dump callback.  Async on the context stream. */
typedef struct {
  int32_t packet, phase;          /* packet index and segment phase (0..2) of the dump */
  gnsscorr_sdr_corr corr;         /* rotated correlations handed to Channel::Accum    */
  gnsscorr_sdr_feedback fb;       /* the NCO_Command_S it returned                    */
} gnsscorr_sdr_dump_rec;          /* 80 bytes */
int gnsscorr_sdr_track_dev(gnsscorr_sdr_corr_ctx *ctx, const int16_t *d_packets, int n_packets,
                           int n_rx, int n_ch, const int32_t *d_rx, gnsscorr_sdr_chan *d_states,
                           gnsscorr_sdr_corr *d_corr, gnsscorr_sdr_channel *d_ch,
                           gnsscorr_sdr_feedback *d_fb_last, gnsscorr_sdr_dump_rec *d_log,
                           int log_per_ch, int32_t *d_n_log, int32_t *d_status,
                           gnsscorr_sdr_subframe *d_events, int max_events,
                           int32_t *d_n_events);

/* ======================================================================
 * GPS-SDR sample front end, bit-exact with
 *   GPS_Source::Read_GN3S   objects/gps_source.cpp:684-767 (2-bit LUT {-3,-1,1,3},
 *                           1024-entry table NCO mix, products truncated to int16)
 *   Resample_GN3S           objects/gps_source.cpp:933-943 (gdec nearest sample)
 *   downsample              accessories/misc.cpp:174-197 (phase-wrap decimator)
 * Output samples are the receivers' CPX (int16 I, Q) at 2.048 Msps, ready for
 * gnsscorr_sdr_acq_strong_dev / gnsscorr_sdr_accum_dev without a host copy.
 * ==================================================================== */
#define GNSSCORR_GN3S_BLOCK_IN  20000          /* 2-bit samples per 5-ms read      */
#define GNSSCORR_GN3S_BLOCK_OUT 10240          /* CPX per 5 ms = 5 packets of 2048 */
#define GNSSCORR_GN3S_STEP      2557223528u    /* delta_phase (gps_source.cpp:96)  */

typedef struct gnsscorr_sdr_fe_ctx gnsscorr_sdr_fe_ctx;

/* The int16 product table the front end uses: out[(code * 1024 + p) * 2 + {0,1}]. */
void gnsscorr_sdr_gn3s_products(int16_t *out);
int gnsscorr_sdr_fe_create(gnsscorr_sdr_fe_ctx **out, int device);
int gnsscorr_sdr_fe_destroy(gnsscorr_sdr_fe_ctx *ctx);
/* n_blocks consecutive 5-ms reads.  fmt 0: one sample per byte (low 2 bits,
 * the reference's gbuff); fmt 1: packed, 4 samples per byte, sample j of a byte
 * in bits 2j..2j+1.  *phase: the NCO phase before the first sample (0 after
 * construction in the reference), advanced by n_blocks * 20000 * step.
 * d_out: n_blocks * 10240 CPX (int16 I, Q), 16-byte aligned (GNSSCORR_EINVAL
 * otherwise).  Asynchronous on the context stream. */
int gnsscorr_sdr_gn3s_dev(gnsscorr_sdr_fe_ctx *ctx, const uint8_t *d_in, int fmt, int n_blocks,
                          uint32_t *phase, uint32_t step, int16_t *d_out);
int gnsscorr_sdr_gn3s(gnsscorr_sdr_fe_ctx *ctx, const uint8_t *h_in, int fmt, int n_blocks,
                      uint32_t *phase, uint32_t step, int16_t *h_out);
/* downsample(): number of samples kept from n_src (and the phase step). */
int gnsscorr_sdr_downsample_count(int n_src, double f_dest, double f_source, uint32_t *step);
/* downsample() of n_src CPX into d_dest (*n_out samples); requires 0 < f_dest < f_source. */
int gnsscorr_sdr_downsample_dev(gnsscorr_sdr_fe_ctx *ctx, const int16_t *d_src, int n_src,
                                double f_dest, double f_source, int16_t *d_dest, int *n_out);
int gnsscorr_sdr_fe_sync(gnsscorr_sdr_fe_ctx *ctx);
void *gnsscorr_sdr_fe_stream(gnsscorr_sdr_fe_ctx *ctx);

/* ======================================================================
 * Device buffers / events (so hosts need no other GPU runtime)
 * ==================================================================== */
int gnsscorr_dev_alloc(int device, size_t bytes, void **d_ptr);
int gnsscorr_dev_free(int device, void *d_ptr);
/* Synchronous copies: each first waits until the device is idle, so they are
 * ordered after every kernel already queued on any context stream. */
int gnsscorr_memcpy_htod(int device, void *d_dst, const void *h_src, size_t bytes);
int gnsscorr_memcpy_dtoh(int device, void *h_dst, const void *d_src, size_t bytes);
int gnsscorr_dev_synchronize(int device);
int gnsscorr_event_create(int device, void **ev);
int gnsscorr_event_record(void *ev, void *stream);
/* Work queued on `stream` after this call waits until `ev` has completed
 * (joins two context streams without a host synchronisation). */
int gnsscorr_stream_wait_event(void *stream, void *ev);
int gnsscorr_event_elapsed_ms(void *start, void *stop, float *ms);
int gnsscorr_event_destroy(void *ev);
/* Fill a device buffer with pseudo-random 2-bit levels {-3,-1,1,3}
 * (benchmark input of the recorded-IF shape; not a signal model). */
int gnsscorr_dev_fill_if2(int device, int8_t *d_buf, size_t bytes, uint64_t seed);

/* ======================================================================
 * Host utilities (deterministic synthetic IF, code tables)
 * ==================================================================== */

/* One planted signal. */
typedef struct {
  int32_t system;         /* 0 = GPS L1 C/A, 1 = GLONASS L1OF (ST code)            */
  int32_t prn;            /* GPS PRN 1..32 (unused for GLONASS)                    */
  int32_t fch;            /* GLONASS frequency channel -7..6                       */
  int32_t data_bits;      /* 1: modulate random 50 bps (GPS) / 100 sym/s (GLO) bits */
  double  code_phase;     /* code phase at sample 0 [chips]                        */
  double  doppler;        /* carrier Doppler [Hz] (code Doppler follows)           */
  double  cn0;            /* C/N0 [dB-Hz]                                          */
  double  carr_phase;     /* carrier phase at sample 0 [rad]                       */
} gnsscorr_sig;

/* Synthetic IF: nsamp complex samples (iq=1: 2*nsamp int8) or real (iq=0),
 * each signal at -(IF + Doppler) in complex baseband (the reference's IQ
 * convention: its wipe-offs multiply by exp(+i 2 pi f t)),
 * at fs with GPS IF `if_gps`, GLONASS IF `if_glo` (+ fch*562.5 kHz), plus
 * complex AWGN, quantised to the 2-bit levels {-3,-1,+1,+3}
 * (gps_source.cpp:692).  Deterministic for a given seed (64-bit LCG). */
int gnsscorr_ifgen(int8_t *h_out, int64_t nsamp, int iq, double fs, double if_gps,
                   double if_glo, int n_sigs, const gnsscorr_sig *sigs, uint64_t seed);

/* GPS C/A code as +-1 chips (generateCAcode.sci:42-87 form), prn 1..32. */
int gnsscorr_ca_code(int prn, int8_t *h_chips1023);
/* GLONASS ST code as +-1 chips (generateSTcode.sci:35-42). */
int gnsscorr_st_code(int8_t *h_chips511);
/* Sample a +-1 chip sequence with the makeCaTable.sci:64-72 rule:
 * out[k-1] = chips[ceil(k*ts/tc)-1], last index forced to code_len. */
int gnsscorr_sample_code(const int8_t *h_chips, int code_len, double code_rate, double fs,
                         int n_samples, int8_t *h_out);

#ifdef __cplusplus
}
#endif
#endif /* GNSSCORR_H */
