// acq_ctx.h -- the acquisition context shared by the fp32 (acq.hip) and the
// reference-precision fp64 (acq64.hip) kernels.  Internal to libgnsscorr.
#ifndef GNSSCORR_ACQ_CTX_H
#define GNSSCORR_ACQ_CTX_H
#include <hip/hip_runtime.h>
#include "gnsscorr_internal.h"

struct gnsscorr_acq_ctx {
  gnsscorr_acq_cfg cfg;
  hipStream_t stream = nullptr;
  int prec = GNSSCORR_ACQ_F64;          // cfg.precision, validated
  // ---- fp32 path (prec == GNSSCORR_ACQ_F32, N = 16368 only)
  int* d_sigma = nullptr;
  float2* d_F = nullptr;     // code spectra, permuted, [max_codes][N]
  float2* d_X = nullptr;     // IF spectra, permuted, [max_freqs*max_blocks][N]
  int4* d_fmap = nullptr;               // per frequency: spectrum class + PFA shift coordinates
  float2* d_stage = nullptr;            // forward-FFT staging rows
  size_t cap_stage = 0;
  int pipe = 1;                         // GNSSCORR_ACQ_PIPE=0: one-unit-per-workgroup kernel
  // ---- fp64 path (prec == GNSSCORR_ACQ_F64)
  int plan64 = 0;                       // acq64 plan id (acq64_plan_for)
  double2* d_F64 = nullptr;             // code spectra, storage order of the plan, [max_codes][rs64]
  double2* d_X64 = nullptr;             // IF class spectra [rows][rs64] (grown per search)
  size_t cap_X64 = 0;
  double2* d_in64 = nullptr;            // natural-order forward-FFT inputs [rows][N] (grown)
  size_t cap_in64 = 0;
  double2* d_twN = nullptr;             // W_N^j, j < N (Cooley-Tukey plans)
  int2* d_fmap64 = nullptr;             // per frequency: {class, shift m mod N}
  int* d_lead64 = nullptr;              // classify scratch: per frequency, its class leader
  int rs64 = 0;                         // fp64 row stride (complex elements)
  // generic-N fp64 plan (plan64 == 3, any other N): Bluestein with radix-16
  // Stockham FFTs of length M = 16^P >= 2N - 1 (acq64.hip)
  int gM = 0, gP = 0;
  double2* d_chirp = nullptr;           // c_n = exp(-i pi n^2 / N), n < N
  double2* d_vf = nullptr;              // FFT_M of the conjugate chirp (two-sided)
  double2* d_twM = nullptr;             // W_M^t, t < M
  double2 *d_gA = nullptr, *d_gB = nullptr;   // chunk x M work rows
  double* d_gpw = nullptr;              // chunk x N power rows
  int g_chunk = 0;                      // rows per chunk
  // mixed-radix Stockham plan of the generic path (N a product of radices in
  // {2..16, 17, 19, 23, 29, 31}; Bluestein otherwise or with GNSSCORR_ACQ_BLUESTEIN=1):
  // mix_nr passes of radix mix_r[i] in global memory, twiddles d_twN (W_N^j)
  int mix_nr = 0;
  int mix_r[24] = {};
  // four-step plan of the generic path (N = N1 N2, N1 = A B and N2 = C D two-radix
  // sub-transforms in LDS, two passes over the rows): 0 none, else its plan index
  int m4 = 0;
  // the four-step plan's per-column top-2 of the power rows (row statistics fused into
  // m4_rows): chunk x N1 entries, or null when the statistics run as their own pass
  void* d_m4top = nullptr;
  double2* d_twm4 = nullptr;            // four-step: W_N1^j (j < N1) then W_N2^j (j < N2)
  // four-step plan, two chunk lanes: odd chunks run on a second stream with their own
  // Y, power rows and column top-2 (m4_lanes == 2), so one chunk's column pass overlaps
  // the other's row pass
  int m4_lanes = 1;
  hipStream_t m4_s2 = nullptr;
  hipEvent_t m4_ev[3] = {nullptr, nullptr, nullptr};   // fork (after lane 0's first column
                                                       // pass), join, spare
  double2* d_gA2 = nullptr;
  double* d_gpw2 = nullptr;
  void* d_m4top2 = nullptr;
  // ---- shared
  int n_codes = 0;
  int spec_blocks = 0, spec_freqs = 0;  // shape of the resident IF spectra
  int* d_order = nullptr;               // workgroup -> work-unit permutation (XCD tiles)
  int order_groups = 0, order_bins = 0, order_units = 0;
  size_t cap_order = 0;
  double* d_cfreq = nullptr;            // per class: the residue frequency whose spectrum is computed
  double* d_resid = nullptr;            // per frequency: its fs/N-grid residue (classify scratch)
  int* d_nclass = nullptr;
  int n_cu = 256;                       // persistent grid of the pipelined kernel
  int coh = 1;                          // code periods per coherent block (set_coherent)
  int recs = 1;                         // records per search (set_records, fp64 plans)
  const int32_t* d_group_rec = nullptr; // per group: its IF record (set_group_records; NULL: every
                                        // group on every record)
  int spec_recs = 1;                    // records of the resident IF spectra
  gnsscorr_acq_row* d_stats = nullptr;  // per (row, block) statistics
  size_t cap_stats = 0;
  int stat_groups = 0, stat_bins = 0, stat_blocks = 0, stat_mode = 0, stat_recs = 1;
  // host-API staging
  int8_t* d_codes8 = nullptr;           // sampled code replicas, int8 [n_codes][N] (grown)
  size_t cap_codes8 = 0;
  int8_t* d_chips = nullptr;            // chip table: rows 0..31 GPS C/A PRN 1..32, row 32 the
                                        // GLONASS ST code (511 chips), 1023 B each (set_prn_codes)
  int8_t* d_if = nullptr;
  double* d_freqs = nullptr;
  int* d_gcode = nullptr;
  int* d_gfreq = nullptr;
  gnsscorr_acq_row* d_rows = nullptr;
  gnsscorr_acq_result* d_res = nullptr;
  double* d_dump = nullptr;
  size_t cap_rows = 0, cap_res = 0, cap_gcode = 0, cap_gfreq = 0;
};

// grow a device buffer to hold `need` elements of `elem` bytes (contents lost)
int acq_grow(void** p, size_t* cap, size_t need, size_t elem);

// ---- acq64.hip: the fp64 engine behind the same context
// plan id for N (0: N not supported by a compiled plan)
int acq64_plan_for(int n_samples);
int acq64_init(gnsscorr_acq_ctx* c);             // device tables for the plan
void acq64_free(gnsscorr_acq_ctx* c);
int acq64_preload(gnsscorr_acq_ctx* c);   // code spectra buffers + code-object load
int acq64_set_codes(gnsscorr_acq_ctx* c, const int8_t* d_codes, int n_codes);
int acq64_spectra(gnsscorr_acq_ctx* c, const int8_t* d_if, int iq, int n_blocks, int n_freqs,
                  const double* d_freqs);
int acq64_correlate(gnsscorr_acq_ctx* c, int n_blocks, int mode, int n_groups, int n_bins,
                    const int32_t* d_gcode, const int32_t* d_gfreq, int spc, double* d_dump,
                    int dump_block);
#endif
