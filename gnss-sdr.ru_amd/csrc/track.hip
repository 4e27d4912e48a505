// track.hip -- GP2021-semantics E/P/L tracking correlator on gfx950.
//
// Replaces the per-sample loop of Sim_GP2021_int
// (reference osgnss_next_step/src/correlator/correlator.c:148-316) with a
// closed-form, sample-parallel formulation that is bit-exact with it:
//
//  * carrier NCO: phase before sample n = P0 + n*cinc (mod 2^32); the 8-phase
//    LO index is its top 3 bits (correlator.c:203-215).
//  * code NCO: rollovers before sample n = (K0 + n*kinc2) >> 32 in 64-bit
//    (kinc2 = code_incr << 1, correlator.c:245), so every thread can start
//    its run of samples anywhere without walking the previous ones.
//  * half-chip / dump logic (correlator.c:246-283) is a function of the
//    rollover count r: until the first dump the half-chip is hc0 + r (uint16);
//    the first dump comes at rollover j1, then every D = slew + 2046
//    rollovers.  The E/P/L bits after the dump rollover are loaded from the
//    PRE-reset index (>= 2046, the reference's row over-read) and half-chip 0
//    of the new epoch keeps them (no reload), which hc_after() reproduces.
//  * accumulation is int32 two's-complement, so per-thread partial sums can
//    be combined in any order: each thread keeps at most two epochs' sums
//    (a run of 64 samples can straddle at most one dump, D >= 2046), the
//    wavefront reduces them with cross-lane shuffles and one lane per wave
//    adds into an LDS slot per epoch.
//
// One workgroup = one channel x one call.  256 threads x 64 samples covers a
// 1-ms chunk at 16.368 Msps; IF is read as 16-byte vector loads.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gnsscorr_internal.h"
#include "if2.h"
#include "osg_isr.h"

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      gnsscorr_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                     \
      return GNSSCORR_EDEVICE;                                                          \
    }                                                                                   \
  } while (0)

// Diagnostic hook (tools/trk_stamps.hip defines it; a no-op in the library)
#ifndef TRACK_PSTAMP
#define TRACK_PSTAMP(i) \
  do {                  \
  } while (0)
#endif

// Diagnostic hook of osg_stream_kernel (tools/trk_stream_stamps.hip; a no-op here)
#ifndef STREAM_PSTAMP
#define STREAM_PSTAMP(i) \
  do {                   \
  } while (0)
#endif

namespace {

constexpr int kRun = 64;              // samples per thread
constexpr int kMaxThreads = 1024;
constexpr int kMaxNsamp = kRun * kMaxThreads;
constexpr uint64_t kNever = ~0ull;
constexpr int kPitch = 9;             // 16-byte chunks per staged lane run (8 + 1 pad)
constexpr int kStageMaxBytes = 48 * 1024;
constexpr int kPk8Stage = 3088;       // LDS bytes of the E/P/L row (D <= 3071: slew <= 1025) + 3 of misalignment
constexpr int kMaxCpw = 4;            // channels per workgroup (32 waves/CU: two 1024-thread WGs)

// 8-phase LO (correlator.c:203-204) as 4-bit two's-complement nibbles.
constexpr uint32_t kLutI = 0xEEF1221Fu;  // i_lo = {-1, 1, 2, 2, 1,-1,-2,-2}
constexpr uint32_t kLutQ = 0x1FEEF122u;  // q_lo = { 2, 2, 1,-1,-2,-2,-1, 1}

struct Chan {
  uint32_t P0, K0, cinc, kinc2, hc0, D;
  uint64_t j1;       // rollover index of the first dump (kNever: none)
  int base;          // prn * 2046 into the packed table
};

// Half-chip counter, table load index and epoch after r rollovers.
__device__ __forceinline__ void hc_after(const Chan& c, uint64_t r, uint32_t& hc, uint32_t& ld,
                                         uint32_t& epoch) {
  if (r < c.j1) {
    epoch = 0;
    hc = (uint32_t)((c.hc0 + r) & 0xFFFFu);
    ld = hc;
  } else {
    uint32_t m = (uint32_t)(r - c.j1);
    epoch = 1 + m / c.D;
    uint32_t q = m % c.D;
    hc = q;
    ld = q ? q : (m == 0 ? (uint32_t)((c.hc0 + c.j1) & 0xFFFFu) : c.D);
  }
}

__device__ __forceinline__ uint32_t n_dumps_after(const Chan& c, uint64_t r) {
  return r >= c.j1 ? 1 + (uint32_t)(r - c.j1) / c.D : 0u;
}

__device__ __forceinline__ void msbit_step(int& ms, int& bit) {
  // correlator.c:275-280
  ms++;
  if (ms == 20) bit = (bit + 1) % 50;
  ms %= 20;
}

// Wave-wide reductions without the LDS crossbar (ds_bpermute): a DPP
// Hillis-Steele scan inside each 16-lane row (row_shr 1/2/4/8, identity
// shifted in), then the four row results (lanes 15/31/47/63) combined in
// scalar registers.  Every lane of the wave must be active.
template <typename Op>
__device__ __forceinline__ int wave_reduce(int v, int ident, Op op) {
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x111, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x112, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x114, 0xF, 0xF, false));
  v = op(v, __builtin_amdgcn_update_dpp(ident, v, 0x118, 0xF, 0xF, false));
  const int a = __builtin_amdgcn_readlane(v, 15), b = __builtin_amdgcn_readlane(v, 31);
  const int c = __builtin_amdgcn_readlane(v, 47), d = __builtin_amdgcn_readlane(v, 63);
  return op(op(a, b), op(c, d));
}
__device__ __forceinline__ int wave_sum(int v) {
  return wave_reduce(v, 0, [](int x, int y) { return (int)((uint32_t)x + (uint32_t)y); });
}
__device__ __forceinline__ int wave_max(int v) {
  return wave_reduce(v, INT_MIN, [](int x, int y) { return max(x, y); });
}
__device__ __forceinline__ int wave_min(int v) {
  return wave_reduce(v, INT_MAX, [](int x, int y) { return min(x, y); });
}

__device__ __forceinline__ int sbyte(int x, int b) { return __builtin_amdgcn_sbfe(x, 8 * b, 8); }

struct Acc {
  uint32_t a[6];
};

template <bool IQ>
__device__ __forceinline__ void corr_sample(int I, int Q, uint32_t& phase, uint32_t& kph,
                                            const Chan& c, uint32_t& hc, int& lb, int& pb,
                                            int& eb, Acc& cur, Acc& first, bool& switched,
                                            const uint32_t* __restrict__ pk) {
  const uint32_t off = (phase >> 27) & 0x1Cu;
  const int il = __builtin_amdgcn_sbfe((int)kLutI, off, 4);
  const int ql = __builtin_amdgcn_sbfe((int)kLutQ, off, 4);
  int ival, qval;
  if (IQ) {
    ival = il * I + ql * Q;   // correlator.c:215
    qval = ql * I - il * Q;   // correlator.c:214
  } else {
    ival = I * il;            // correlator.c:222-223
    qval = I * ql;
  }
  cur.a[0] += (uint32_t)(lb * ival);
  cur.a[1] += (uint32_t)(lb * qval);
  cur.a[2] += (uint32_t)(pb * ival);
  cur.a[3] += (uint32_t)(pb * qval);
  cur.a[4] += (uint32_t)(eb * ival);
  cur.a[5] += (uint32_t)(eb * qval);
  phase += c.cinc;
  const uint32_t nk = kph + c.kinc2;
  const bool carry = nk < kph;
  kph = nk;
  if (carry) {
    hc = (hc + 1u) & 0xFFFFu;
    const uint32_t ld = hc;
    if (hc >= c.D) {  // dump (correlator.c:251-281)
#pragma unroll
      for (int k = 0; k < 6; k++) { first.a[k] = cur.a[k]; cur.a[k] = 0; }
      switched = true;
      hc = 0;
    }
    const uint32_t w = pk[c.base + (int)ld];
    lb = (int)(int8_t)(w & 0xFFu);
    pb = (int)(int8_t)((w >> 8) & 0xFFu);
    eb = (int)(int8_t)((w >> 16) & 0xFFu);
  }
}

// ---- IQ fast path: segment sums with v_dot4 ---------------------------------
// Between two code-NCO carries (one half-chip, ~8 samples) the E/P/L bits are
// constant, so acc_X += bit_X * ival(n) over the segment equals bit_X times the
// segment sum S = sum ival(n) (int32 wrap keeps it exact).  ival/qval of a
// pair of samples (n, n+1) is ONE v_dot4_i32_i8 of the IF word {I0,Q0,I1,Q1}
// with the LO word {il(a), ql(a), il(b), ql(b)} resp. {ql(a), -il(a), ql(b),
// -il(b)} (correlator.c:213-215), a / b the 8-phase LO indices of the two
// samples; the 64 (a, b) LO word pairs sit in LDS.  A carry between the two
// samples splits the pair with byte masks.
__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// |segment sum| < 2^23 and bits are -1/0/+1: the 24-bit multiply is exact
// (int32 wrap on the accumulator, as the reference).  __mul24 (llvm.amdgcn.mul.i24)
// + add is selected as v_mad_i32_i24; a plain `c + a * b` becomes a 64-bit
// v_mad_u64_u32.  This used to be an inline-asm v_mad_i32_i24: an INLINEASM
// carries no implicit EXEC operand, so machine passes were free to move it
// across the exec-mask writes of divergent branches, where it then wrote
// lanes of a reused register that the branch had masked off -- the cause of
// the wrong sums DESIGN.md recorded for reordered IF loads in round 2.
__device__ __forceinline__ uint32_t mad24(int a, int b, uint32_t c) {
  return c + (uint32_t)__mul24(a, b);
}
__device__ __forceinline__ void seg_flush(int si, int sq, int lb, int pb, int eb, Acc& cur) {
  cur.a[0] = mad24(lb, si, cur.a[0]);
  cur.a[1] = mad24(lb, sq, cur.a[1]);
  cur.a[2] = mad24(pb, si, cur.a[2]);
  cur.a[3] = mad24(pb, sq, cur.a[3]);
  cur.a[4] = mad24(eb, si, cur.a[4]);
  cur.a[5] = mad24(eb, sq, cur.a[5]);
}

// E/P/L bits of one half-chip as three 2-bit two's-complement fields
// (late | prompt << 2 | early << 4; values -1 / 0 / +1), see pack8_table()
__device__ __forceinline__ void unpack8(uint32_t w, int& lb, int& pb, int& eb) {
  lb = __builtin_amdgcn_sbfe((int)w, 0, 2);
  pb = __builtin_amdgcn_sbfe((int)w, 2, 2);
  eb = __builtin_amdgcn_sbfe((int)w, 4, 2);
}

// the carry branch of correlator.c:243-283 (half-chip step, dump, bit reload);
// tb: the channel's packed E/P/L row (LDS-staged, or the global table + base)
template <typename TB>
__device__ __forceinline__ void code_carry(const Chan& c, uint32_t& hc, int& lb, int& pb, int& eb,
                                           Acc& cur, Acc& first, bool& switched, TB tb) {
  hc = (hc + 1u) & 0xFFFFu;
  const uint32_t ld = hc;
  if (hc >= c.D) {
#pragma unroll
    for (int k = 0; k < 6; k++) { first.a[k] = cur.a[k]; cur.a[k] = 0; }
    switched = true;
    hc = 0;
  }
  unpack8(tb[ld], lb, pb, eb);
}

// one sample (the odd last sample of a tail run): x = {I, Q, 0, 0}
template <typename TB>
__device__ __forceinline__ void corr_single(uint32_t x, uint32_t& p0, uint32_t& kph, const Chan& c,
                                            uint32_t& hc, int& lb, int& pb, int& eb, int& si,
                                            int& sq, Acc& cur, Acc& first, bool& switched,
                                            const uint2* __restrict__ lo2, TB tb) {
  const uint2 lo = lo2[p0 >> 29];
  p0 += c.cinc;
  si = dot4(x, lo.x & 0xFFFFu, si);
  sq = dot4(x, lo.y & 0xFFFFu, sq);
  const uint32_t k0 = kph + c.kinc2;
  const bool c0 = k0 < kph;
  kph = k0;
  if (c0) {
    seg_flush(si, sq, lb, pb, eb, cur);
    code_carry(c, hc, lb, pb, eb, cur, first, switched, tb);
    si = 0;
    sq = 0;
  }
}

// samples n0, n0+1 (IF word x), carrier phases p0 / p0 + cinc
template <typename TB>
__device__ __forceinline__ void corr_pair(uint32_t x, uint32_t& p0, uint32_t& kph, const Chan& c,
                                          uint32_t& hc, int& lb, int& pb, int& eb, int& si,
                                          int& sq, Acc& cur, Acc& first, bool& switched,
                                          const uint2* __restrict__ lo2, TB tb) {
  const uint32_t p1 = p0 + c.cinc;
  const uint2 lo = lo2[(p0 >> 29) | ((p1 >> 26) & 0x38u)];
  p0 = p1 + c.cinc;
  const uint32_t k0 = kph + c.kinc2;
  const uint32_t k1 = k0 + c.kinc2;
  const bool c0 = k0 < kph, c1 = k1 < k0;
  kph = k1;
  if (!(c0 | c1)) {   // no code carry in the pair (3 of 4 pairs at 8 samples/half-chip)
    si = dot4(x, lo.x, si);
    sq = dot4(x, lo.y, sq);
    return;
  }
  if (!c0) {
    si = dot4(x, lo.x, si);
    sq = dot4(x, lo.y, sq);
  } else {   // carry after the first sample of the pair
    si = dot4(x, lo.x & 0xFFFFu, si);
    sq = dot4(x, lo.y & 0xFFFFu, sq);
    seg_flush(si, sq, lb, pb, eb, cur);
    code_carry(c, hc, lb, pb, eb, cur, first, switched, tb);
    si = dot4(x, lo.x & 0xFFFF0000u, 0);
    sq = dot4(x, lo.y & 0xFFFF0000u, 0);
  }
  if (c1) {
    seg_flush(si, sq, lb, pb, eb, cur);
    code_carry(c, hc, lb, pb, eb, cur, first, switched, tb);
    si = 0;
    sq = 0;
  }
}

// Per-channel epilogue of a call (one thread): dumps, ms/bit counters, TIC latch,
// carrier cycles and the new channel state (correlator.c:243-316).  sum(i):
// the call's epoch sums, word i = epoch * 6 + k (LDS or global).  st_out (if
// given) receives the new state as well.
template <typename SumAt>
__device__ __forceinline__ gnsscorr_track_result channel_epilogue(
    const Chan& c, const gnsscorr_nco_cmd& cmd, gnsscorr_chan_state st, int chn, bool active,
    uint32_t ndump, uint64_t Rtot, int nsamp, int64_t tic_count, SumAt sum,
    gnsscorr_track_result* __restrict__ res, gnsscorr_chan_state* __restrict__ state,
    int32_t* __restrict__ all_dumps, int max_dumps, gnsscorr_chan_state* st_out = nullptr) {
  if (!active) {   // idle channel: only the epoch load (correlator.c:177-185)
    gnsscorr_track_result r;
    memset(&r, 0, sizeof r);
    r.n_dumps = cmd.prn > 32 ? -1 : 0;
    r.msbit_reg = st.msbit_reg;
    res[chn] = r;
    state[chn] = st;
    if (st_out) *st_out = st;
    return r;
  }
  gnsscorr_track_result r;
  memset(&r, 0, sizeof r);
  r.n_dumps = (int)ndump;
  int ms = st.ms_counter, bit = st.bit_counter, msbit = st.msbit_reg;

  const bool tic_here = tic_count >= 0 && tic_count < nsamp;
  uint32_t nd_tic = 0;
  uint64_t Rt = 0;
  if (tic_here) {
    Rt = ((uint64_t)c.K0 + (uint64_t)(tic_count + 1) * c.kinc2) >> 32;
    nd_tic = n_dumps_after(c, Rt);
  }
  int msbit_at_tic = msbit;
  for (uint32_t d = 0; d < ndump; d++) {
    uint32_t v[6];
#pragma unroll
    for (int k = 0; k < 6; k++)
      v[k] = sum(d * 6 + k) + (d == 0 ? (uint32_t)st.acc[k] : 0u);
    if (all_dumps && (int)d < max_dumps)
      for (int k = 0; k < 6; k++) all_dumps[((int64_t)chn * max_dumps + d) * 6 + k] = (int32_t)v[k];
    if (d + 1 == ndump)
      for (int k = 0; k < 6; k++) r.dump[k] = (int32_t)v[k];
    msbit_step(ms, bit);
    msbit = ms + (bit << 8);
    if (d + 1 == nd_tic) msbit_at_tic = msbit;
  }
  uint32_t nacc[6];
  for (int k = 0; k < 6; k++)
    nacc[k] = sum(ndump * 6 + k) + (ndump == 0 ? (uint32_t)st.acc[k] : 0u);

  const uint64_t Wtot = ((uint64_t)c.P0 + (uint64_t)nsamp * c.cinc) >> 32;
  uint32_t cycle_end;
  if (tic_here) {  // TIC latch after sample tic_count (correlator.c:286-303)
    const uint64_t t1 = (uint64_t)tic_count + 1;
    const uint64_t Wt = ((uint64_t)c.P0 + t1 * c.cinc) >> 32;
    const uint32_t cyc = st.carrier_cycle + (uint32_t)Wt;
    uint32_t hct, ldt, ept;
    hc_after(c, Rt, hct, ldt, ept);
    r.tic = 1;
    r.tic_regs[0] = (int32_t)hct;
    r.tic_regs[1] = (int32_t)(cyc & 0xffffu);
    r.tic_regs[2] = (int32_t)((c.P0 + (uint32_t)t1 * c.cinc) >> 22);
    r.tic_regs[3] = msbit_at_tic;
    r.tic_regs[4] = (int32_t)((uint32_t)((uint64_t)c.K0 + t1 * c.kinc2) >> 22);
    r.tic_regs[5] = (int32_t)(cyc >> 16);
    cycle_end = (uint32_t)(Wtot - Wt);
  } else {
    cycle_end = st.carrier_cycle + (uint32_t)Wtot;
  }
  uint32_t hce, lde, epe;
  hc_after(c, Rtot, hce, lde, epe);

  r.msbit_reg = msbit;
  res[chn] = r;

  st.carrier_phase = c.P0 + (uint32_t)nsamp * c.cinc;
  st.carrier_cycle = cycle_end;
  st.code_phase = (uint32_t)((uint64_t)c.K0 + (uint64_t)nsamp * c.kinc2);
  st.half_chip = hce;
  for (int k = 0; k < 6; k++) st.acc[k] = (int32_t)nacc[k];
  st.ms_counter = ms;
  st.bit_counter = bit;
  st.msbit_reg = msbit;
  state[chn] = st;
  if (st_out) *st_out = st;
  return r;
}

// Epoch-segmented reduction of the per-thread sums and the per-channel epilogue
// (one thread per channel): dumps, ms/bit counters, TIC latch, carrier cycles and
// the new channel state (correlator.c:243-316).  Every thread of the workgroup
// calls it (it holds a barrier).
__device__ __forceinline__ void finish_call(const Chan& c, const gnsscorr_nco_cmd& cmd,
                                            gnsscorr_chan_state st, int chn, bool have,
                                            bool active, int tid, bool runs, int e0,
                                            bool switched, const Acc& first, const Acc& cur,
                                            int32_t* s_sum, uint32_t ndump, uint64_t Rtot,
                                            int nsamp, int64_t tic_count,
                                            gnsscorr_track_result* __restrict__ res,
                                            gnsscorr_chan_state* __restrict__ state,
                                            int32_t* __restrict__ all_dumps, int max_dumps) {
  // ---- epoch-segmented reduction ------------------------------------------
  // thread contributes (e0, switched ? first : cur) and (e0+1, cur) if switched
  // (a wave never spans two thread groups: T is a multiple of 64)
  const int e_hi_mine = e0 + (switched ? 1 : 0);
  const int e_lo = wave_min(runs ? e0 : 0x7fffffff);
  const int e_hi = wave_max(runs ? e_hi_mine : -1);
  const int lane = threadIdx.x & 63;
  for (int e = e_lo; e <= e_hi; e++) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
      uint32_t v = 0;
      if (e == e0) v += switched ? first.a[k] : cur.a[k];
      if (switched && e == e0 + 1) v += cur.a[k];
      const int s = wave_sum((int)v);
      if (lane == 0) atomicAdd(&s_sum[e * 6 + k], s);
    }
  }
  __syncthreads();
  TRACK_PSTAMP(4);

  // ---- per-channel epilogue (one thread per channel) ------------------------
  if (tid != 0 || !have) return;
  channel_epilogue(c, cmd, st, chn, active, ndump, Rtot, nsamp, tic_count,
                   [&](int i) { return (uint32_t)s_sum[i]; }, res, state, all_dumps, max_dumps);
  TRACK_PSTAMP(5);
}

__device__ __forceinline__ int xcd_channel(int b, int G) {
  const int q = G >> 3, r = G & 7, x = b & 7, slot = b >> 3;
  return x * q + (x < r ? x : r) + slot;
}

// ============================================================================
// osg_track2_kernel: branch-free segment sums for interleaved I,Q streams
// (int8 or 2-bit packed).
//
// Why: in osg_track_kernel every lane walks its own 64-sample run and takes a
// code-carry branch about once per 8 samples, at a different sample in every
// lane, so a wave executes the carry path (segment flush, bit reload, epoch
// switch) at nearly every sample pair: ~18 VALU + ~12 SALU instructions per
// sample (PMC, round 2).  Here a lane's samples are cut into intervals of
// three pairs (6 samples).  When a half-chip lasts at least 6 samples (kinc2 <=
// 2^32 / 6, any fs >= 12.3 Msps) an interval holds at most one code carry, so
// every pair is split branch-free into the part before the carry ("pre", LO
// word masked by the carry position) and the whole pair ("tot"); at the end of
// each interval -- the same instruction for every lane -- the pre sums are
// flushed with the current E/P/L bits (correlator.c:213-241), the remainder
// carries over into the next segment and the bits are reloaded once
// (correlator.c:243-251).  The rare dump (epoch switch, correlator.c:251-281)
// is the only branch.
//
// Sample -> lane map: wave w of a channel covers samples [4096 w, 4096 w + 4096)
// as two pieces of 2048; lane l takes samples [2048 p + 32 l, +32) of piece p.
// A piece is 64 lanes x 32 samples of CONTIGUOUS IF, so each wave load reads
// 1 KiB of consecutive bytes: int8 pieces (4 KiB) are staged through a
// wave-private LDS slot (no workgroup barrier), packed pieces (16 B per lane)
// are loaded straight into registers and expanded with v_perm.  No IF is
// shared between channels, so the receiver layout (12 channels per stream)
// and one stream per channel run the same code with the same LDS footprint.
//
// Channels outside the fast path's conditions (kinc2 > 2^32/6, a half-chip
// range beyond the staged E/P/L row, no dump possible) run the per-sample
// reference recurrence (corr_sample) on the same staged words, wave-uniformly.
// ============================================================================
constexpr int kPieceLen = 32;                    // samples per lane per piece
constexpr int kPieceSpan = 64 * kPieceLen;       // samples per wave per piece
constexpr int kWaveSpan = 2 * kPieceSpan;        // samples per wave
constexpr int kStage2Bytes = kPieceSpan * 2;     // int8 IQ bytes of one staged piece (4 KiB)
constexpr uint32_t kFastKinc2 = 0xFFFFFFFFu / 6u;   // >= 6 samples per half-chip

// hc_after without a 32-bit division (m < 2^24: fp32 reciprocal + one fix-up)
__device__ __forceinline__ void hc_after_fast(const Chan& c, uint64_t r, float invD, uint32_t& hc,
                                              uint32_t& ld, uint32_t& epoch) {
  if (r < c.j1) {
    epoch = 0;
    hc = (uint32_t)((c.hc0 + r) & 0xFFFFu);
    ld = hc;
  } else {
    const uint32_t m = (uint32_t)(r - c.j1);
    uint32_t e = (uint32_t)((float)m * invD);
    // e < 2^14 and D < 2^17 (r counts the half-chips of one call): a full-rate
    // 24-bit multiply, not v_mul_lo_u32
    int q = (int)(m - __umul24(e, c.D));
    if (q < 0) { q += (int)c.D; e--; }
    if (q >= (int)c.D) { q -= (int)c.D; e++; }
    epoch = 1 + e;
    hc = (uint32_t)q;
    ld = q ? (uint32_t)q : (m == 0 ? (uint32_t)((c.hc0 + c.j1) & 0xFFFFu) : c.D);
  }
}

// Lane state through its pieces.
struct Seg {
  uint32_t p0, kph, hc, ld;
  uint32_t cb, nb;             // TRACK_PF: row byte of the current bits / of index hc + 1
  int lb, pb, eb;
  int ti, tq, pi, pq;          // interval sums: whole pairs / part before the carry
  bool carried;               // a code carry in the current interval
};

// one pair of samples (IF word x) in the branch-free interval form; ONE: the
// word holds a single (last) sample, so no carry after a second one
template <bool ONE>
__device__ __forceinline__ void pair2(uint32_t x, const Chan& c, Seg& g, const uint2* __restrict__ lo2) {
  const uint32_t p1 = g.p0 + c.cinc;
  const uint2 lo = lo2[(g.p0 >> 29) | ((p1 >> 26) & 0x38u)];
  g.p0 = p1 + c.cinc;
  const uint32_t k0 = g.kph + c.kinc2;
  const bool c0 = k0 < g.kph;
  uint32_t k1 = k0;
  bool c1 = false;
  if (!ONE) {
    k1 = k0 + c.kinc2;
    c1 = k1 < k0;
  }
  g.kph = k1;
  uint32_t m = c0 ? 0xFFFFu : 0xFFFFFFFFu;   // carry after sample a: only a is "pre"
  m = g.carried ? 0u : m;                    // after this interval's carry: nothing is
  g.carried = g.carried | c0 | c1;
  const uint32_t xm = x & m;
  g.ti = dot4(x, lo.x, g.ti);
  g.tq = dot4(x, lo.y, g.tq);
  g.pi = dot4(xm, lo.x, g.pi);
  g.pq = dot4(xm, lo.y, g.pq);
}

// pair2 with the LO word pairs as two 256-byte tables (ival words, qval words):
// a ds_read_b32 of 64 lanes then touches each bank at most once per distinct
// entry (64 entries x 4 B = the 64 banks), where the 512-byte uint2 table put
// entries e and e + 32 on the same banks
template <bool ONE>
__device__ __forceinline__ void pair2s(uint32_t x, const Chan& c, Seg& g,
                                       const uint32_t* __restrict__ lox,
                                       const uint32_t* __restrict__ loy) {
  const uint32_t p1 = g.p0 + c.cinc;
  const uint32_t idx = (g.p0 >> 29) | ((p1 >> 26) & 0x38u);
  const uint32_t lo_x = lox[idx], lo_y = loy[idx];
  g.p0 = p1 + c.cinc;
  const uint32_t k0 = g.kph + c.kinc2;
  const bool c0 = k0 < g.kph;
  uint32_t k1 = k0;
  bool c1 = false;
  if (!ONE) {
    k1 = k0 + c.kinc2;
    c1 = k1 < k0;
  }
  g.kph = k1;
  uint32_t m = c0 ? 0xFFFFu : 0xFFFFFFFFu;
  m = g.carried ? 0u : m;
  g.carried = g.carried | c0 | c1;
  const uint32_t xm = x & m;
  g.ti = dot4(x, lo_x, g.ti);
  g.tq = dot4(x, lo_y, g.tq);
  g.pi = dot4(xm, lo_x, g.pi);
  g.pq = dot4(xm, lo_y, g.pq);
}

// end of an interval: flush the part before the carry with the current bits,
// carry the rest into the next segment, step the half-chip (correlator.c:243-283)
__device__ __forceinline__ void interval_end(const Chan& c, Seg& g, Acc& cur, Acc& first,
                                             bool& switched, const uint8_t* __restrict__ row) {
  seg_flush(g.pi, g.pq, g.lb, g.pb, g.eb, cur);
  const int ri = g.ti - g.pi, rq = g.tq - g.pq;
  g.ti = g.pi = ri;
  g.tq = g.pq = rq;
  const bool cy = g.carried;               // branch-free: one carry at most
  g.hc += cy ? 1u : 0u;
  g.ld = cy ? g.hc : g.ld;
  g.carried = false;
  // (a half-chip count already >= D -- slew lowered between calls -- dumps at
  // the next carry, not before: the reference tests only after a step)
  if (cy && g.hc >= c.D) {   // dump (correlator.c:251-281): rare, one lane per channel
    // snapshot of the epoch's sums; cur keeps running over both epochs and the
    // lane's share of the next epoch is cur - first (osg_track2_kernel's end)
#pragma unroll
    for (int k = 0; k < 6; k++) first.a[k] = cur.a[k];
    switched = true;
    g.hc = 0;          // the bits of half-chip 0 come from the pre-reset index ld
  }
  unpack8(row[g.ld], g.lb, g.pb, g.eb);
}

// The per-wave piece path (see the osg_track2 notes above): every lane's two
// 32-sample pieces in the branch-free interval form (fast) or by the per-sample
// recurrence; sums as (old epoch, new epoch) in (first, cur) when switched.
// s_wave: this wave's 4 KiB LDS slot (int8 streams).
template <bool PK>
__device__ __forceinline__ void run_pieces(const int8_t* __restrict__ ifbuf, int64_t stream_stride,
                                           int nsamp, int tid, const Chan& c, int stream,
                                           bool active, bool fast, const uint8_t* s_pk8,
                                           const uint2* s_lo, uint4* s_wave,
                                           const uint32_t* __restrict__ pk, Acc& cur, Acc& first,
                                           bool& switched, int& e0, bool& runs) {
  const float invD = 1.0f / (float)c.D;
  const int lane = (int)threadIdx.x & 63;
  const int wbase = (tid >> 6) * kWaveSpan;               // first sample of this wave
  runs = active && wbase + lane * kPieceLen < nsamp;
  // element offset of the channel's stream
  const int64_t e_stream = (int64_t)stream * stream_stride * 2;
  Seg g;

#pragma unroll
  for (int p = 0; p < 2; p++) {
    const int n_piece = wbase + p * kPieceSpan;            // first sample of the wave's piece
    if (!active || n_piece >= nsamp) break;                // wave-uniform
    const int n0 = n_piece + lane * kPieceLen;             // this lane's first sample
    const int L = max(0, min(kPieceLen, nsamp - n0));      // this lane's valid samples
    // ---- IF of the lane's piece: 16 sample-pair words in 4 chunks of 4
    uint32_t pw[4] = {0u, 0u, 0u, 0u};   // packed: one 32-bit word (4 pairs) per chunk
    if constexpr (PK) {
      // 16 B per lane (8-byte aligned streams): two 8-byte loads of whole bytes
      const uint8_t* b = reinterpret_cast<const uint8_t*>(ifbuf) + ((e_stream + 2 * (int64_t)n0) >> 2);
      if (L == kPieceLen) {
        const uint2 u0 = reinterpret_cast<const uint2*>(b)[0];
        const uint2 u1 = reinterpret_cast<const uint2*>(b)[1];
        pw[0] = u0.x; pw[1] = u0.y; pw[2] = u1.x; pw[3] = u1.y;
      } else {
        for (int k = 0; 2 * k < L; k++) pw[k >> 2] |= (uint32_t)b[k] << (8 * (k & 3));
      }
    } else {
      // int8: the wave's 4 KiB piece through its LDS slot.  Chunk i (16 B) of the
      // piece belongs to lane i >> 2; it is stored at lane * 64 + 16 * ((i ^ (lane >> 2)) & 3)
      // so that the 16-byte reads of 16 consecutive lanes hit 64 distinct banks.
      const int8_t* g8 = ifbuf + e_stream + 2 * (int64_t)n_piece;
      const int valid = max(0, min(kPieceSpan, nsamp - n_piece));   // samples of the piece in the call
      const int full_chunks = valid / 8;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int i = r * 64 + lane;
        const int ow = i >> 2, sub = i & 3;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (i < full_chunks) {
          v = reinterpret_cast<const uint4*>(g8)[i];
        } else if (i * 8 < valid) {   // the partial chunk: whole words, then the odd sample
          const int rem = valid - i * 8;   // 1..7 samples
          const uint32_t* g32 = reinterpret_cast<const uint32_t*>(g8) + 4 * i;
          uint32_t t[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int k = 0; k < 3; k++)
            if (k < rem / 2) t[k] = g32[k];
          const uint32_t odd = (rem & 1) ? (uint32_t)reinterpret_cast<const uint16_t*>(g32)[rem - 1] : 0u;
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (k == rem / 2) t[k] = odd;
          v = make_uint4(t[0], t[1], t[2], t[3]);
        }
        s_wave[ow * 4 + ((sub ^ (ow >> 2)) & 3)] = v;
      }
      __builtin_amdgcn_wave_barrier();
    }
    // chunk j of the lane's piece as four pair words
    auto chunk = [&](int j) -> uint4 {
      if constexpr (PK) return if2_expand_word(pw[j]);
      else return s_wave[lane * 4 + ((j ^ (lane >> 2)) & 3)];
    };
    if (L > 0) {
      // ---- lane state at its first sample
      const uint64_t X = (uint64_t)c.K0 + (uint64_t)n0 * c.kinc2;
      const uint64_t r0 = X >> 32;
      g.kph = (uint32_t)X;
      if (fast) {
        // closed form at the piece start; a dump between the lane's two pieces
        // shows as a later epoch (at most one dump per lane: D >= 2046 half-chips)
        uint32_t ep;
        hc_after_fast(c, r0, invD, g.hc, g.ld, ep);
        if (p == 0) {
          e0 = (int)ep;
        } else if ((int)ep > e0 + (switched ? 1 : 0)) {
#pragma unroll
          for (int k = 0; k < 6; k++) first.a[k] = cur.a[k];   // snapshot (see interval_end)
          switched = true;
        }
        unpack8(s_pk8[g.ld], g.lb, g.pb, g.eb);
        g.ti = g.tq = g.pi = g.pq = 0;
        g.carried = false;
        // one code path per wave: a wave with one partial lane (the call's last
        // samples) runs the guarded loop for all its lanes instead of both loops
        if (__all(L == kPieceLen)) {   // every wave but the last of a channel
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint4 u = chunk(j);
            const uint32_t words[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int k = 4 * j + i;
              pair2<false>(words[i], c, g, s_lo);
              if (k % 3 == 2 || k == kPieceLen / 2 - 1) interval_end(c, g, cur, first, switched, s_pk8);
            }
          }
        } else {
          const int np = L >> 1;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint4 u = chunk(j);
            const uint32_t words[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int k = 4 * j + i;
              if (k < np) pair2<false>(words[i], c, g, s_lo);
              else if (k == np && (L & 1)) pair2<true>(words[i] & 0xFFFFu, c, g, s_lo);
              if (k % 3 == 2 || k == kPieceLen / 2 - 1) interval_end(c, g, cur, first, switched, s_pk8);
            }
          }
        }
        // the samples after the piece's last carry: the open segment, with the
        // bits in force after it
        seg_flush(g.ti, g.tq, g.lb, g.pb, g.eb, cur);
      } else {
        // per-sample reference recurrence (correlator.c:200-283), table from global memory
        uint32_t hc, ld, ep;
        hc_after(c, r0, hc, ld, ep);
        if (p == 0) {
          e0 = (int)ep;
        } else if ((int)ep > e0 + (switched ? 1 : 0)) {
#pragma unroll
          for (int k = 0; k < 6; k++) first.a[k] = cur.a[k];   // snapshot
          switched = true;
        }
        const uint32_t tw = pk[c.base + (int)ld];
        int lb = (int)(int8_t)(tw & 0xFFu), pb = (int)(int8_t)((tw >> 8) & 0xFFu),
            eb = (int)(int8_t)((tw >> 16) & 0xFFu);
        // corr_sample keeps (first, cur) as (old epoch, new epoch); the kernel
        // keeps (snapshot, running total): convert around the call
        if (switched)
#pragma unroll
          for (int k = 0; k < 6; k++) cur.a[k] -= first.a[k];
        uint32_t phase = g.p0, kph = g.kph;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint4 u = chunk(j);
          const uint32_t words[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int k = 4 * j + i;
#pragma unroll
            for (int h = 0; h < 2; h++)
              if (2 * k + h < L)
                corr_sample<true>(sbyte((int)words[i], 2 * h), sbyte((int)words[i], 2 * h + 1), phase,
                                  kph, c, hc, lb, pb, eb, cur, first, switched, pk);
          }
        }
        if (switched)
#pragma unroll
          for (int k = 0; k < 6; k++) cur.a[k] += first.a[k];
      }
    }
    if constexpr (!PK) __builtin_amdgcn_wave_barrier();   // the slot is refilled by the next piece
  }
  if (switched)   // (snapshot, running total) -> (old epoch, new epoch) for finish_call
#pragma unroll
    for (int k = 0; k < 6; k++) cur.a[k] -= first.a[k];
}


// One workgroup = cpw channels (cpw = 1024 / threads-per-channel, at most
// kMaxCpw) x one call; thread group q = threadIdx.x / T runs channel
// grp*cpw + q.  When every active channel of the workgroup reads the same IF
// stream (the channels of one receiver), the stream's 64-sample runs are
// staged once in LDS with coalesced 16-byte loads and shared by the cpw
// channels: each lane's run would otherwise be 8 loads that put every lane on
// its own cache line (8x the L2 -> CU bytes, once per channel).
// PK: the IF streams are GNSSCORR_IF_PACKED2 (if2.h): staged runs are expanded
// to int8 in LDS; unstaged runs expand per 16-element word in registers.
template <bool IQ, bool PK>
__global__ __launch_bounds__(kMaxThreads, 8) void osg_track_kernel(
    const int8_t* __restrict__ ifbuf, int64_t stream_stride, int nsamp, int n_channels, int cpw,
    const gnsscorr_nco_cmd* __restrict__ cmds, gnsscorr_chan_state* __restrict__ state,
    gnsscorr_track_result* __restrict__ res, int32_t* __restrict__ all_dumps, int max_dumps,
    const uint32_t* __restrict__ pk, const uint8_t* __restrict__ pk8, int64_t tic_count,
    int stage_ok) {
  __shared__ uint2 s_lo[64];
  __shared__ int s_stream[kMaxCpw];
  __shared__ int s_short[kMaxCpw];
  // dynamic LDS: [cpw][ep_cap][6] epoch sums | [cpw][kPk8Stage] E/P/L row bytes |
  // staged IF runs (lane runs of 128 B at a 144 B pitch)
  extern __shared__ uint4 s_dyn[];
  const int ep_cap = nsamp / GNSSCORR_OSG_ROW + 2;   // >= epochs of one call
  const int sum_words = ((cpw * ep_cap * 6) + 3) & ~3;
  const int T = (int)blockDim.x / cpw;
  // wave-uniform (T is a multiple of 64): keeps the channel's command, state
  // and NCO constants in scalar registers
  const int q = __builtin_amdgcn_readfirstlane((int)threadIdx.x / T);
  const int tid = (int)threadIdx.x - q * T;
  int32_t* s_sum = reinterpret_cast<int32_t*>(s_dyn) + q * ep_cap * 6;
  uint8_t* s_pk8 = reinterpret_cast<uint8_t*>(s_dyn) + sum_words * 4 + q * kPk8Stage;
  uint4* s_if = s_dyn + sum_words / 4 + cpw * (kPk8Stage / 16);
  // XCD-aware order: workgroup b runs on XCD b % 8, so give every XCD a
  // contiguous channel range -- the channels of one receiver (consecutive
  // channels sharing an IF stream) then hit the same 4 MiB L2 and the stream
  // is fetched from HBM once instead of once per XCD.
  TRACK_PSTAMP(0);
  const int chn = xcd_channel(blockIdx.x, gridDim.x) * cpw + q;
  const bool have = chn < n_channels;
  gnsscorr_nco_cmd cmd = {};
  gnsscorr_chan_state st = {};
  if (have) {
    cmd = cmds[chn];
    st = state[chn];
  }
  if (cmd.epoch_load >= 0) {  // epoch set, correlator.c:177-182
    const int v = cmd.epoch_load & 0xFFFF;
    st.msbit_reg = v;
    st.ms_counter = v & 0xff;
    st.bit_counter = v >> 8;
  }
  const bool active = have && cmd.prn > 0 && cmd.prn <= 32;   // correlator.c:185
  if (tid == 0) s_stream[q] = active ? cmd.stream : -1;

  Chan c;
  c.P0 = st.carrier_phase;
  c.K0 = st.code_phase;
  c.cinc = cmd.carrier_incr;
  c.kinc2 = cmd.code_incr << 1;
  c.hc0 = st.half_chip & 0xFFFFu;
  c.D = (cmd.slew & 0xFFFFu) + 2046u;
  {
    const uint32_t h1 = (c.hc0 + 1u) & 0xFFFFu;
    if (h1 >= c.D) c.j1 = 1;
    else if (c.D <= 0xFFFFu) c.j1 = 1ull + (c.D - h1);
    else c.j1 = kNever;  // uint16 half-chip can never reach D
  }
  c.base = (active ? cmd.prn : 0) * GNSSCORR_OSG_ROW;
  // A lane of the piece path covers kPieceSpan + kPieceLen samples (two pieces)
  // and holds at most one dump.  Two consecutive dumps are D code carries
  // apart, at least D * 2^32 / kinc2 - 1 samples: a channel whose epoch can be
  // that short (about 2.05-2.08 Msps, one half-chip per sample) sends its
  // workgroup to the per-thread 64-sample runs, which hold one dump at most.
  if (tid == 0)
    s_short[q] = active && ((uint64_t)c.D << 32) <= (uint64_t)(kPieceSpan + kPieceLen + 1) * c.kinc2;
  TRACK_PSTAMP(1);
  const uint64_t Rtot = ((uint64_t)c.K0 + (uint64_t)nsamp * c.kinc2) >> 32;
  const uint32_t ndump = n_dumps_after(c, Rtot);
  const int n_epochs = (int)ndump + 1;

  if (active)
    for (int i = tid; i < n_epochs * 6; i += T) s_sum[i] = 0;
  if (IQ && threadIdx.x < 64) {   // LO words of the sample pair (a, b) = (t & 7, t >> 3)
    const int a = threadIdx.x & 7, b = threadIdx.x >> 3;
    const uint32_t ia = (uint32_t)__builtin_amdgcn_sbfe((int)kLutI, 4 * a, 4) & 0xFFu;
    const uint32_t qa = (uint32_t)__builtin_amdgcn_sbfe((int)kLutQ, 4 * a, 4) & 0xFFu;
    const uint32_t ib = (uint32_t)__builtin_amdgcn_sbfe((int)kLutI, 4 * b, 4) & 0xFFu;
    const uint32_t qb = (uint32_t)__builtin_amdgcn_sbfe((int)kLutQ, 4 * b, 4) & 0xFFu;
    s_lo[threadIdx.x] = make_uint2(ia | qa << 8 | ib << 16 | qb << 24,
                                   qa | ((0u - ia) & 0xFFu) << 8 | qb << 16 | ((0u - ib) & 0xFFu) << 24);
  }
  // The half-chip table indices of this call lie in [0, max(D, hc0, hc0+1)]
  // (correlator.c:243-251; the dump reloads from the pre-reset index D):
  // stage that part of the channel's row in LDS so the reload at every code
  // carry is an LDS read, not a dependent global-memory round trip.
  const uint32_t pk_hi = max(max(c.D, c.hc0), (c.hc0 + 1u) & 0xFFFFu);
  const bool pk_lds = IQ && active && c.j1 != kNever && pk_hi < 3072u;
  if (pk_lds) {
    // whole dwords of the row (the packed table is padded by 64 bytes): byte i of
    // the staged row is s_pk8[i] with s_pk8 offset by the row's misalignment
    const uint32_t* g32 = reinterpret_cast<const uint32_t*>(pk8) + (c.base >> 2);
    uint32_t* l32 = reinterpret_cast<uint32_t*>(s_pk8);
    const int n32 = (int)((pk_hi + (uint32_t)(c.base & 3)) >> 2) + 1;
    for (int i = tid; i < n32; i += T) l32[i] = g32[i];
  }
  s_pk8 += c.base & 3;
  __syncthreads();
  int sst = -1;
  bool uni = true, any_short = false;
  for (int k = 0; k < cpw; k++) {
    const int v = s_stream[k];
    any_short |= s_short[k] != 0;
    if (v >= 0) {
      if (sst < 0) sst = v;
      else if (v != sst) uni = false;
    }
  }
  // stage_ok: 0 no staging (lanes read their runs from global memory); 1 a
  // stream shared by the whole workgroup is staged once in LDS and read by its
  // cpw channels; channels of a workgroup on different streams (one stream
  // per channel, receivers split over workgroups) take the per-wave piece
  // path (run_pieces: coalesced 1 KiB wave loads, no workgroup barrier)
  // (stage_ok 4: A/B, the piece path for every workgroup)
  const bool shared_stage = IQ && stage_ok && stage_ok != 4 && uni && sst >= 0;
  const bool pieces = IQ && (stage_ok == 1 || stage_ok == 4) && !shared_stage && !any_short;
  const bool stage = shared_stage;
  uint4* s_ifq = s_if;
  if (stage) {
    const int n_full = nsamp / kRun;
    const int st_id = sst;
    const int lt = (int)threadIdx.x;       // staging lane and width
    const int nt = (int)blockDim.x;
    uint32_t* t32 = reinterpret_cast<uint32_t*>(s_ifq + n_full * kPitch);
    if constexpr (!PK) {
      // full 64-sample runs only; consecutive threads load consecutive 16-byte chunks
      const int4* g = reinterpret_cast<const int4*>(ifbuf + (int64_t)st_id * stream_stride * 2);
      const int n_chunks = n_full * (kRun * 2 / 16);
      for (int ch = lt; ch < n_chunks; ch += nt) {
        const int4 v = g[ch];
        s_ifq[(ch >> 3) * kPitch + (ch & 7)] = make_uint4(v.x, v.y, v.z, v.w);
      }
      // the whole sample pairs of the tail run go to the next slot (an odd last
      // sample is read from global memory by its lane)
      const uint32_t* g32 = reinterpret_cast<const uint32_t*>(g) + n_full * (kRun / 2);
      for (int wi = lt; wi < (nsamp - n_full * kRun) / 2; wi += nt) t32[wi] = g32[wi];
    } else {
      // packed: one byte per sample pair; an 8-byte chunk (packed data is
      // only 8-byte aligned: 1 ms at 16.368 Msps is 8184 bytes) is a quarter
      // run and expands to two 16-byte int8 chunks (once per workgroup,
      // shared by its cpw channels)
      const uint8_t* gb = reinterpret_cast<const uint8_t*>(ifbuf) + (int64_t)st_id * stream_stride / 2;
      const uint2* g = reinterpret_cast<const uint2*>(gb);
      const int n_chunks = n_full * 4;
      for (int ch = lt; ch < n_chunks; ch += nt) {
        const uint2 v = g[ch];
        uint4* d = &s_ifq[(ch >> 2) * kPitch + (ch & 3) * 2];
        d[0] = if2_expand_word(v.x);
        d[1] = if2_expand_word(v.y);
      }
      for (int wi = lt; wi < (nsamp - n_full * kRun) / 2; wi += nt)
        t32[wi] = if2_expand_byte(gb[n_full * (kRun / 2) + wi]);
    }
    __syncthreads();
  }
  TRACK_PSTAMP(2);

  Acc cur, first;
#pragma unroll
  for (int k = 0; k < 6; k++) { cur.a[k] = 0; first.a[k] = 0; }
  bool switched = false;
  int e0 = 0;
  bool runs = false;
  if (pieces) {
    // the fast (branch-free) form needs the row in LDS and >= 6 samples per half-chip
    const bool fast = pk_lds && c.kinc2 <= kFastKinc2;
    const int wave = (int)threadIdx.x >> 6;
    run_pieces<PK>(ifbuf, stream_stride, nsamp, tid, c, cmd.stream, active, fast, s_pk8, s_lo,
                   s_if + wave * (kStage2Bytes / 16), pk, cur, first, switched, e0, runs);
  } else {
  // ---- per-thread run of kRun samples --------------------------------------
  const int n0 = tid * kRun;
  runs = active && n0 < nsamp;
  if (runs) {
    const uint64_t X = (uint64_t)c.K0 + (uint64_t)n0 * c.kinc2;
    uint32_t kph = (uint32_t)X;
    uint32_t phase = c.P0 + (uint32_t)n0 * c.cinc;
    uint32_t hc, ld, ep;
    hc_after(c, X >> 32, hc, ld, ep);
    e0 = (int)ep;
    int lb, pb, eb;
    if (pk_lds) {
      unpack8(s_pk8[ld], lb, pb, eb);
    } else {
      const uint32_t w = pk[c.base + (int)ld];
      lb = (int)(int8_t)(w & 0xFFu);
      pb = (int)(int8_t)((w >> 8) & 0xFFu);
      eb = (int)(int8_t)((w >> 16) & 0xFFu);
    }
    constexpr int kBps = IQ ? 2 : 1;
    // element offset of the run (a multiple of 64: n0 and the stream base are);
    // src is its first byte in either format
    const int64_t e_run = ((int64_t)cmd.stream * stream_stride + n0) * kBps;
    const int8_t* src = PK ? ifbuf + (e_run >> 2) : ifbuf + e_run;
    const uint8_t* srcb = reinterpret_cast<const uint8_t*>(src);
    // {I, Q} word of sample k of the run (odd last sample of a tail run)
    auto single_word = [&](int k) -> uint32_t {
      if constexpr (PK)
        return (if2_expand_byte(srcb[k >> 1]) >> (16 * (k & 1))) & 0xFFFFu;
      else
        return (uint32_t)srcb[2 * k] | (uint32_t)srcb[2 * k + 1] << 8;
    };
    if (IQ && pk_lds) {   // (a channel whose half-chip range exceeds the staged row takes
                          //  the per-sample path below, reading the table from global memory)
      constexpr int kVec = kRun * 2 / 16;
      const int L = min(kRun, nsamp - n0);
      auto body = [&](auto tb) {
        int si = 0, sq = 0;
        const int np = L >> 1;
        // one 16-byte int8 chunk = 4 sample pairs (chunk j of the run)
        auto chunk = [&](const uint4 u, int j) {
          const uint32_t words[4] = {u.x, u.y, u.z, u.w};
          if (4 * j + 4 <= np) {
#pragma unroll
            for (int wd = 0; wd < 4; wd++)
              corr_pair(words[wd], phase, kph, c, hc, lb, pb, eb, si, sq, cur, first, switched,
                        s_lo, tb);
          } else {
            for (int wd = 0; wd < 4; wd++)
              if (4 * j + wd < np)
                corr_pair(words[wd], phase, kph, c, hc, lb, pb, eb, si, sq, cur, first, switched,
                          s_lo, tb);
          }
        };
        if (stage || (!PK && L == kRun)) {
          // one 16-byte chunk (4 pairs) per iteration with the next one in
          // flight: a rolled loop keeps the register footprint small enough
          // for two 1024-thread workgroups per CU.  The tail run (staged in
          // LDS) goes through the same loop with its missing pairs masked, so
          // it does not serialise behind the full runs of its wave.
          {
          // one loop per source, typed by address space: a pointer selected
          // between the LDS stage and global memory is a generic pointer, and
          // its loads became flat loads, which count in both vmcnt and lgkmcnt -- every wait for a
          // LO-word or E/P/L-row read then also waited for the prefetch
          typedef unsigned int V4U __attribute__((ext_vector_type(4)));
          auto run_loop = [&](auto run) {
            V4U nx = run[0];
#pragma unroll 1
            for (int j = 0; j < kVec; j++) {
              const uint4 u = make_uint4(nx.x, nx.y, nx.z, nx.w);
              if (j + 1 < kVec) nx = run[j + 1];
              chunk(u, j);
            }
          };
          typedef const __attribute__((address_space(3))) V4U* LdsU4;
          typedef const __attribute__((address_space(1))) V4U* GlbU4;
          if (stage)
            run_loop((LdsU4)(&s_ifq[tid * kPitch]));
          else
            run_loop((GlbU4)(src));
          }
        } else if (PK && L == kRun) {
          // packed, unstaged (channels of a workgroup on different streams):
          // the run is 32 bytes (8-byte aligned), each 4-byte word expands
          // to one int8 chunk
          const uint2* prun = reinterpret_cast<const uint2*>(src);
          uint2 nx = prun[0];
#pragma unroll 1
          for (int h = 0; h < 4; h++) {
            const uint2 p = nx;
            if (h + 1 < 4) nx = prun[h + 1];
            chunk(if2_expand_word(p.x), 2 * h);
            chunk(if2_expand_word(p.y), 2 * h + 1);
          }
        } else {   // tail run without staging (one lane): same arithmetic, word loads
          const uint32_t* w32 = reinterpret_cast<const uint32_t*>(src);
          for (int k = 0; k < np; k++)
            corr_pair(PK ? if2_expand_byte(srcb[k]) : w32[k], phase, kph, c, hc, lb, pb, eb, si,
                      sq, cur, first, switched, s_lo, tb);
        }
        if (L & 1)
          corr_single(single_word(L - 1), phase, kph, c, hc, lb, pb, eb, si, sq, cur, first,
                      switched, s_lo, tb);
        seg_flush(si, sq, lb, pb, eb, cur);
      };
      body(s_pk8);
    } else if (!PK && n0 + kRun <= nsamp) {
      const int4* v = reinterpret_cast<const int4*>(src);
      constexpr int kVec = kRun * kBps / 16;
#pragma unroll
      for (int j = 0; j < kVec; j++) {
        const int4 q = v[j];
        const int words[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int wd = 0; wd < 4; wd++) {
          const int x = words[wd];
          if (IQ) {
            corr_sample<IQ>(sbyte(x, 0), sbyte(x, 1), phase, kph, c, hc, lb, pb, eb, cur, first,
                            switched, pk);
            corr_sample<IQ>(sbyte(x, 2), sbyte(x, 3), phase, kph, c, hc, lb, pb, eb, cur, first,
                            switched, pk);
          } else {
#pragma unroll
            for (int b = 0; b < 4; b++)
              corr_sample<IQ>(sbyte(x, b), 0, phase, kph, c, hc, lb, pb, eb, cur, first,
                              switched, pk);
          }
        }
      }
    } else {   // per sample (tail runs; every packed run off the fast path)
      const int L = min(kRun, nsamp - n0);
      for (int k = 0; k < L; k++) {
        const int I = if_elem(src, (int64_t)k * kBps, PK);
        const int Q = IQ ? if_elem(src, (int64_t)k * kBps + 1, PK) : 0;
        corr_sample<IQ>(I, Q, phase, kph, c, hc, lb, pb, eb, cur, first, switched, pk);
      }
    }
  }

  }   // per-thread runs
  TRACK_PSTAMP(3);
  finish_call(c, cmd, st, chn, have, active, tid, runs, e0, switched, first, cur, s_sum, ndump, Rtot,
              nsamp, tic_count, res, state, all_dumps, max_dumps);
}



// ============================================================================
// osg_stream_kernel: ONE WAVEFRONT PER CHANNEL AND CALL (interleaved I,Q
// streams, int8 or 2-bit packed; round 4).
//
// The wave walks its channel's call in pieces of 2048 samples (lane l takes
// the contiguous samples [2048 p + 32 l, +32) of piece p), with the next
// piece already on its way while the current one is correlated:
//   * int8: LDS-DMA (global_load_lds_dwordx4, 4 wave-instructions of 1 KiB of
//     consecutive IF each) into the wave's 4 KiB slot; after the piece has
//     landed the lanes copy their 64 bytes to registers and the DMA of the
//     next piece is issued into the same slot;
//   * packed: the lane's 16 bytes straight into registers, one piece ahead.
// Each piece runs the branch-free interval form of run_pieces (pair2 /
// interval_end: at most one code carry per 6 samples) when a half-chip lasts
// >= 6 samples and the channel's E/P/L row fits the LDS stage, else the
// per-sample reference recurrence.  A lane carries ONE set of six running sums
// (its current epoch) across all its pieces; at an epoch change -- a dump
// inside its samples, or a later piece that starts in a later epoch -- it adds
// them into the wave's per-epoch LDS sums with LDS atomics (behind a
// wave-uniform branch: dumps are rare) and starts over.  No cross-lane
// reduction and no workgroup barrier: the epoch sums are complete when the
// wave is, and lane 0 runs the channel's epilogue (correlator.c:243-316).
//
// Against the per-call workgroup kernel (4 waves of 64-sample lanes per
// channel): the per-wave fixed work (reduction, epilogue, state setup) is
// paid once per channel-call instead of four times, the IF of the next piece
// streams in while the current one computes, and a lane holds at most one
// dump per piece (32 samples << D >= 2046 half-chips) at every sample rate.
// Channels sharing a stream (receivers) read it through L2, which the
// XCD-aware channel order keeps on one XCD.
// ============================================================================
#ifndef TRACK_STREAM_CH
#define TRACK_STREAM_CH 4
#endif
constexpr int kStreamCh = TRACK_STREAM_CH;   // channels (wavefronts) per workgroup
#ifndef TRACK_PF
#define TRACK_PF 1                // LO words and row bytes read ahead (pair2r, interval_end_s)
#endif
#ifndef TRACK_NODUMP_COPY
#define TRACK_NODUMP_COPY 1       // pieces without a dump run a copy without the dump test
#endif
#ifndef TRACK_IV4
#define TRACK_IV4 1               // 4-pair intervals when a half-chip lasts >= 8 samples
#endif
#ifndef TRACK_ALIGNED
#define TRACK_ALIGNED 1           // pieces whose code carries repeat every 8 samples: fixed masks
#endif
#ifndef TRACK_X2LUT
#define TRACK_X2LUT 1             // packed bytes expanded through a 256-word LDS table
#endif
constexpr uint32_t kIv4Kinc2 = 0x20000000u;   // 8 kinc2 <= 2^32

// The int8 piece slot (4 KiB: 256 chunks of 16 B = 8 IQ samples; lane l's 32
// samples are chunks 4 l .. 4 l + 3) is swizzled: chunk g sits at entry
// slot_entry(g) = 4 (g / 4) + ((g % 4) XOR (g / 16 % 4)).  A lane's ds_read_b128
// of its chunk j then hits 16-byte bank slot 4 (l % 4) + (j XOR (l / 4 % 4)), and
// each of the instruction's four 16-lane groups ({0-3,12-15,20-27}, ...,
// MI355X_MICROARCH.md LDS table) holds four lanes of every l % 4 with four
// different l / 4 % 4: 16 distinct slots, conflict-free.  Unswizzled, the lanes'
// 64-byte stride put four lanes on every slot (4-way, 12 extra LDS cycles per
// read).  The map is its own inverse: DMA entry e is
// filled from chunk slot_entry(e), which stays inside e's 4-chunk group, so a
// DMA instruction still reads whole 128-byte lines.
__device__ __forceinline__ int slot_entry(int g) { return g ^ ((g >> 4) & 3); }
__device__ __forceinline__ int slot_chunk(int e) { return slot_entry(e); }

// Orders LDS accesses between the lanes of ONE wave: every lane's earlier LDS
// writes (plain stores and atomics) are visible to every lane's later LDS reads
// and atomics.  The wave executes its LDS instructions in order, but without a
// fence the compiler may move one lane's read above another lane's write: the
// per-thread memory model knows nothing of the other lanes (the
// round-4 state broadcast bug).  Wavefront-scope fences emit no instruction; the
// wave barrier keeps the scheduler from moving memory operations across.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void flush_epoch(Acc& acc, int e, int32_t* s_sum) {
#pragma unroll
  for (int k = 0; k < 6; k++) {
    atomicAdd(&s_sum[e * 6 + k], (int)acc.a[k]);
    acc.a[k] = 0;
  }
}

// Adds the six sums of every lane in `fl` (its epoch: e) into the wave's per-epoch
// LDS sums and, with CLEAR, zeroes them.  Per distinct epoch among those lanes
// (almost always one) a DPP scan inside each 16-lane row, then one LDS atomic per
// row from lanes 15/31/47/63.  Every lane of the wave must be active.  The piece
// starts after a dump and the call's end flush most lanes at once: 64 lanes each
// adding to the same six words serialise on one LDS address (63 extra LDS cycles
// per atomic, the bulk of the kernel's SQ_LDS_BANK_CONFLICT).
template <bool CLEAR>
__device__ __forceinline__ void flush_lanes(bool fl, Acc& acc, int e, int32_t* s_sum, int lane) {
  uint64_t m = __builtin_amdgcn_ballot_w64(fl);
  asm volatile("" : "+s"(m));
  while (m) {
    const int E = __builtin_amdgcn_readlane(e, (int)__builtin_ctzll(m));
    const bool mine = fl && e == E;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      int v = mine ? (int)acc.a[k] : 0;
      v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
      v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
      if ((lane & 15) == 15) atomicAdd(&s_sum[E * 6 + k], v);
      if (CLEAR) acc.a[k] = mine ? 0u : acc.a[k];
    }
    uint64_t done = __builtin_amdgcn_ballot_w64(mine);
    asm volatile("" : "+s"(done));
    m &= ~done;
  }
}

// LDS per wavefront: [IF slot (int8)] [E/P/L row] [epoch sums] [64 LO word pairs]
__host__ __device__ constexpr int stream_sum_bytes(int nsamp) {
  return (((nsamp / GNSSCORR_OSG_ROW + 2) * 24 + 15) & ~15);
}
__host__ __device__ constexpr int stream_wave_lds(bool pk, int nsamp) {
  return (pk ? 0 : kStage2Bytes) + kPk8Stage + stream_sum_bytes(nsamp) + 512;
}

// Arguments of one osg_stream_kernel launch: n_calls consecutive calls of
// every channel (replay or closed loop) or one call.
struct StreamArgs {
  const int8_t* ifbuf;
  int64_t stream_stride;      // samples
  int64_t call_elems;         // int8 elements of one call within a stream (call k at + k*call_elems)
  int nsamp, n_channels, n_calls, cmd_step;   // call k's commands: cmds + k*cmd_step
  gnsscorr_nco_cmd* cmds;
  gnsscorr_chan_state* state;
  gnsscorr_track_result* res;  // call k: res + k*n_channels
  int32_t* all_dumps;          // single calls only
  int max_dumps;
  const uint32_t* pk;
  const uint8_t* pk8;
  int64_t tic, tic_ref;        // tic_explicit: call 0's TIC sample; else the TIC counter
  int tic_explicit;            // before call 0, stepped as gnsscorr_track_next_tic does
  int xcall_prefetch;          // prefetch the next call's first piece during this call's last
  gnsscorr_osg_loop_cfg lk;    // closed loop (loops != nullptr): gpsisr after every call
  gnsscorr_osg_loop* loops;
  gnsscorr_osg_loop* hist;     // call k: hist + k*n_channels (optional)
};

// interval end (see interval_end): flush the part before the carry, carry the
// rest, step the half-chip; a dump adds the epoch's sums to the LDS and
// starts the next epoch
template <bool PF, bool DUMPS = true>
__device__ __forceinline__ void interval_end_s(const Chan& c, Seg& g, Acc& acc, int& e,
                                               int32_t* s_sum, const uint8_t* __restrict__ row) {
  seg_flush(g.pi, g.pq, g.lb, g.pb, g.eb, acc);
  const int ri = g.ti - g.pi, rq = g.tq - g.pq;
  g.ti = g.pi = ri;
  g.tq = g.pq = rq;
  const bool cy = g.carried;
  g.hc += cy ? 1u : 0u;
  if constexpr (!PF) g.ld = cy ? g.hc : g.ld;
  g.carried = false;
  if constexpr (DUMPS) {   // (!DUMPS: the caller showed that no lane dumps in this piece)
    const bool dump = cy && g.hc >= c.D;   // correlator.c:251-281
    uint64_t any = __builtin_amdgcn_ballot_w64(dump);
    asm volatile("" : "+s"(any));          // a uniform branch: the flush stays off the common path
    if (any) {
      if (dump) {
        flush_epoch(acc, e, s_sum);
        e++;
        g.hc = 0;        // the bits of half-chip 0 come from the pre-reset index ld
      }
    }
  }
  if constexpr (PF) {
    // a carry moves to index hc + 1 (the pre-reset index when it dumps): its row
    // byte was read one interval ahead; the next one is read now
    g.cb = cy ? g.nb : g.cb;
    unpack8(g.cb, g.lb, g.pb, g.eb);
    g.nb = row[g.hc + 1];
  } else {
    unpack8(row[g.ld], g.lb, g.pb, g.eb);
  }
}

// pair2s with the pair's LO words already in registers (TRACK_PF: a piece's 16
// LO word pairs are read from LDS before its first interval)
template <bool ONE>
__device__ __forceinline__ void pair2r(uint32_t x, uint32_t lo_x, uint32_t lo_y, const Chan& c,
                                       Seg& g) {
  const uint32_t k0 = g.kph + c.kinc2;
  const bool c0 = k0 < g.kph;
  uint32_t k1 = k0;
  bool c1 = false;
  if (!ONE) {
    k1 = k0 + c.kinc2;
    c1 = k1 < k0;
  }
  g.kph = k1;
  uint32_t m = c0 ? 0xFFFFu : 0xFFFFFFFFu;
  m = g.carried ? 0u : m;
  g.carried = g.carried | c0 | c1;
  const uint32_t xm = x & m;
  g.ti = dot4(x, lo_x, g.ti);
  g.tq = dot4(x, lo_y, g.tq);
  g.pi = dot4(xm, lo_x, g.pi);
  g.pq = dot4(xm, lo_y, g.pq);
}

// one sample of the reference recurrence (correlator.c:200-283) on the
// running sums; ROW: the E/P/L bits from the LDS row, else the global table
template <bool ROW>
__device__ __forceinline__ void corr_sample_s(int I, int Q, uint32_t& phase, uint32_t& kph,
                                              const Chan& c, uint32_t& hc, int& lb, int& pb,
                                              int& eb, Acc& acc, int& e, int32_t* s_sum,
                                              const uint8_t* row, const uint32_t* __restrict__ pk) {
  const uint32_t off = (phase >> 27) & 0x1Cu;
  const int il = __builtin_amdgcn_sbfe((int)kLutI, off, 4);
  const int ql = __builtin_amdgcn_sbfe((int)kLutQ, off, 4);
  const int ival = il * I + ql * Q;   // correlator.c:215
  const int qval = ql * I - il * Q;   // correlator.c:214
  acc.a[0] += (uint32_t)(lb * ival);
  acc.a[1] += (uint32_t)(lb * qval);
  acc.a[2] += (uint32_t)(pb * ival);
  acc.a[3] += (uint32_t)(pb * qval);
  acc.a[4] += (uint32_t)(eb * ival);
  acc.a[5] += (uint32_t)(eb * qval);
  phase += c.cinc;
  const uint32_t nk = kph + c.kinc2;
  const bool carry = nk < kph;
  kph = nk;
  if (carry) {
    hc = (hc + 1u) & 0xFFFFu;
    const uint32_t ld = hc;
    if (hc >= c.D) {
      flush_epoch(acc, e, s_sum);
      e++;
      hc = 0;
    }
    if constexpr (ROW) {
      unpack8(row[ld], lb, pb, eb);
    } else {
      const uint32_t w = pk[c.base + (int)ld];
      lb = (int)(int8_t)(w & 0xFFu);
      pb = (int)(int8_t)((w >> 8) & 0xFFu);
      eb = (int)(int8_t)((w >> 16) & 0xFFu);
    }
  }
}

// channel state and NCO words of one call (correlator.c:177-189)
__device__ __forceinline__ bool chan_setup(const gnsscorr_nco_cmd& cmd, gnsscorr_chan_state& st,
                                           Chan& c) {
  if (cmd.epoch_load >= 0) {  // epoch set, correlator.c:177-182
    const int v = cmd.epoch_load & 0xFFFF;
    st.msbit_reg = v;
    st.ms_counter = v & 0xff;
    st.bit_counter = v >> 8;
  }
  const bool active = cmd.prn > 0 && cmd.prn <= 32;   // correlator.c:185
  c.P0 = st.carrier_phase;
  c.K0 = st.code_phase;
  c.cinc = cmd.carrier_incr;
  c.kinc2 = cmd.code_incr << 1;
  c.hc0 = st.half_chip & 0xFFFFu;
  c.D = (cmd.slew & 0xFFFFu) + 2046u;
  const uint32_t h1 = (c.hc0 + 1u) & 0xFFFFu;
  if (h1 >= c.D) c.j1 = 1;
  else if (c.D <= 0xFFFFu) c.j1 = 1ull + (c.D - h1);
  else c.j1 = kNever;
  c.base = (active ? cmd.prn : 0) * GNSSCORR_OSG_ROW;
  return active;
}

// Open loop: at least 4 waves per SIMD (<= 128 VGPRs; the build takes 117, no
// spills): 3072 channels put 3 waves on a SIMD, 12288 put 4; same-box A/B
// 3 % faster than the unbounded build at 3072 channels.  The closed loop (gpsisr
// inlined, ~150 VGPRs) keeps the default bound.
#ifndef TRACK_STREAM_WAVES
#define TRACK_STREAM_WAVES 4
#endif
template <bool PK, bool CLOSED>
__global__ __launch_bounds__(64 * kStreamCh, CLOSED ? 1 : TRACK_STREAM_WAVES) void osg_stream_kernel(
    StreamArgs A) {
  // the LO words read ahead (TRACK_PF) in the open loop only: in the closed loop
  // their 32 registers pushed the kernel from 151 to 183 VGPRs (2 waves per SIMD:
  // 32.6 -> 42.7 us per 3072-channel call, same box)
  constexpr bool kPF = TRACK_PF && !CLOSED;
  extern __shared__ uint4 s_dyn[];
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int lane = (int)threadIdx.x & 63;
  const int nsamp = A.nsamp;
  const int ep_cap = nsamp / GNSSCORR_OSG_ROW + 2;
  // the 64 (a, b) LO word pairs as two 256-byte tables at a fixed LDS address,
  // shared by the workgroup's waves: a pair's words are one ds_read2_b32 whose
  // address is the byte index 4 (a | b << 3) itself (kPF); without the read-ahead
  // each wave keeps its own copy beside its sums (s_lo)
  __shared__ uint32_t s_lot[128];
  // packed: byte b -> its four int8 levels (one LDS read instead of the spread
  // and v_perm of if2_expand_byte per output word)
  constexpr bool kX2 = PK && TRACK_X2LUT;
  __shared__ uint32_t s_x2[kX2 ? 256 : 1];
  if constexpr (kX2) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_x2[i] = if2_expand_byte((uint32_t)i);
  }
  if (kPF && threadIdx.x < 64) {
    const int a = lane & 7, b = lane >> 3;
    const uint32_t ia = (uint32_t)__builtin_amdgcn_sbfe((int)kLutI, 4 * a, 4) & 0xFFu;
    const uint32_t qa = (uint32_t)__builtin_amdgcn_sbfe((int)kLutQ, 4 * a, 4) & 0xFFu;
    const uint32_t ib = (uint32_t)__builtin_amdgcn_sbfe((int)kLutI, 4 * b, 4) & 0xFFu;
    const uint32_t qb = (uint32_t)__builtin_amdgcn_sbfe((int)kLutQ, 4 * b, 4) & 0xFFu;
    s_lot[lane] = ia | qa << 8 | ib << 16 | qb << 24;
    s_lot[64 + lane] = qa | ((0u - ia) & 0xFFu) << 8 | qb << 16 | ((0u - ib) & 0xFFu) << 24;
  }
  if (kPF || kX2) __syncthreads();   // the only workgroup barrier: before any wave leaves
  uint8_t* wb = reinterpret_cast<uint8_t*>(s_dyn) + wave * stream_wave_lds(PK, nsamp);
  uint4* const slot = reinterpret_cast<uint4*>(wb);                // int8 only: the piece slot
  uint8_t* s_row = wb + (PK ? 0 : kStage2Bytes);
  int32_t* s_sum = reinterpret_cast<int32_t*>(s_row + kPk8Stage);
  uint2* s_lo = reinterpret_cast<uint2*>(reinterpret_cast<uint8_t*>(s_sum) + stream_sum_bytes(nsamp));
  STREAM_PSTAMP(0);
  const int C = A.n_channels;
  const int chn = xcd_channel(blockIdx.x, gridDim.x) * kStreamCh + wave;
  if (chn >= C) return;   // wave-uniform; no workgroup barrier from here on
  if constexpr (!kPF) {
    const int a = lane & 7, b = lane >> 3;   // LO words of the sample pair (a, b)
    const uint32_t ia = (uint32_t)__builtin_amdgcn_sbfe((int)kLutI, 4 * a, 4) & 0xFFu;
    const uint32_t qa = (uint32_t)__builtin_amdgcn_sbfe((int)kLutQ, 4 * a, 4) & 0xFFu;
    const uint32_t ib = (uint32_t)__builtin_amdgcn_sbfe((int)kLutI, 4 * b, 4) & 0xFFu;
    const uint32_t qb = (uint32_t)__builtin_amdgcn_sbfe((int)kLutQ, 4 * b, 4) & 0xFFu;
    uint32_t* lt = reinterpret_cast<uint32_t*>(s_lo);
    lt[lane] = ia | qa << 8 | ib << 16 | qb << 24;
    lt[64 + lane] = qa | ((0u - ia) & 0xFFu) << 8 | qb << 16 | ((0u - ib) & 0xFFu) << 24;
  }
  const uint32_t* lox = reinterpret_cast<const uint32_t*>(s_lo);
  const uint32_t* loy = lox + 64;
  (void)lox;
  (void)loy;
  constexpr bool closed = CLOSED;   // A.loops != nullptr: gpsisr after every call
  gnsscorr_chan_state st = A.state[chn];
  gnsscorr_nco_cmd cmd = A.cmds[chn];
  int64_t tic = A.tic;
  const int n_pieces = (nsamp + kPieceSpan - 1) / kPieceSpan;
  int row_base = -1, row_n32 = 0;   // the E/P/L row words staged in s_row (uniform)

  // ---- the piece in flight: LDS-DMA into the wave's slot (int8), or the lane's
  // 16 bytes in registers (packed).  iss / con: pieces issued / consumed; (q_k,
  // q_p): the last issued.
  int iss = 0, con = 0, q_k = -1, q_p = -1;
  uint2 pq0 = make_uint2(0u, 0u), pq1 = make_uint2(0u, 0u);
  auto issue = [&](int k, int p, int64_t e_call) {   // e_call: element offset of call k's stream
    const int n_piece = p * kPieceSpan;
    if constexpr (PK) {
      const int n0 = n_piece + lane * kPieceLen;
      const uint8_t* b = reinterpret_cast<const uint8_t*>(A.ifbuf) + ((e_call + 2 * (int64_t)n0) >> 2);
      if (n0 + kPieceLen <= nsamp) {
        pq0 = reinterpret_cast<const uint2*>(b)[0];
        pq1 = reinterpret_cast<const uint2*>(b)[1];
      } else {
        const int L = max(0, nsamp - n0);
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        for (int q = 0; 2 * q < L; q++) w[q >> 2] |= (uint32_t)b[q] << (8 * (q & 3));
        pq0 = make_uint2(w[0], w[1]);
        pq1 = make_uint2(w[2], w[3]);
      }
    } else {
      const int valid = min(kPieceSpan, nsamp - n_piece);
      const int full_chunks = valid / 8;
      const int8_t* g8 = A.ifbuf + e_call + 2 * (int64_t)n_piece;
      // DMA instruction r writes slot entries 64 r + lane; it reads the chunk the
      // entry holds in the swizzled slot layout (slot_chunk: the chunks of one
      // 128-byte line stay within one 8-lane group, so the loads stay coalesced)
      if (full_chunks == kPieceSpan / 8) {   // a whole piece: no per-lane guards
#pragma unroll
        for (int r = 0; r < 4; r++)
          __builtin_amdgcn_global_load_lds(
              (const void*)(g8 + 16 * slot_chunk(r * 64 + lane)),
              (__attribute__((address_space(3))) void*)(slot + r * 64), 16, 0, 0);
      } else {
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int i = slot_chunk(r * 64 + lane);
          if (i < full_chunks)
            __builtin_amdgcn_global_load_lds(
                (const void*)(g8 + 16 * i),
                (__attribute__((address_space(3))) void*)(slot + r * 64), 16, 0, 0);
        }
      }
    }
    iss = __builtin_amdgcn_readfirstlane(iss + 1);   // (uniform: scalar registers)
    q_k = __builtin_amdgcn_readfirstlane(k);
    q_p = __builtin_amdgcn_readfirstlane(p);
  };

  for (int k = 0; k < A.n_calls; k++) {
    // TIC of this call (gnsscorr_track_next_tic, correlator.c:155-165)
    int64_t tic_k;
    if (A.tic_explicit) {
      tic_k = tic;
    } else if (tic < nsamp) {
      tic_k = tic;
      tic += A.tic_ref - nsamp;
    } else {
      tic -= nsamp;
      tic_k = -1;
    }
    if (k > 0 && !closed) cmd = A.cmds[(int64_t)k * A.cmd_step + chn];
    Chan c;
    const bool active = chan_setup(cmd, st, c);
    const int64_t e_call = (int64_t)cmd.stream * A.stream_stride * 2 + (int64_t)k * A.call_elems;
    wave_lds_sync();   // lane 0 read the previous call's sums: they are zeroed only after
    for (int i = lane; i < ep_cap * 6; i += 64) s_sum[i] = 0;
    wave_lds_sync();   // ... and every lane's flushes add to zeroed sums
    const uint32_t pk_hi = max(max(c.D, c.hc0), (c.hc0 + 1u) & 0xFFFFu);
    const bool pk_lds = active && c.j1 != kNever && pk_hi < 3072u;
    if (active && q_k != k) issue(k, 0, e_call);
    if (pk_lds) {
      // the staged row serves later calls of the same PRN (replay, closed loop)
      // as far as it reaches
      const int n32 = (int)((pk_hi + (uint32_t)(c.base & 3)) >> 2) + 1;
      if (c.base != row_base || n32 > row_n32) {
        const uint32_t* g32 = reinterpret_cast<const uint32_t*>(A.pk8) + (c.base >> 2);
        uint32_t* l32 = reinterpret_cast<uint32_t*>(s_row);
        for (int i = lane; i < n32; i += 64) l32[i] = g32[i];
        row_base = c.base;
        row_n32 = n32;
      }
      wave_lds_sync();   // lanes read row words other lanes staged
    }
    STREAM_PSTAMP(1);
    const uint8_t* row = s_row + (c.base & 3);
    const bool fast = pk_lds && c.kinc2 <= kFastKinc2;
    const float invD = 1.0f / (float)c.D;
    // the next call's first piece (prefetched during this call's last piece)
    int64_t e_next = -1;
    if (k + 1 < A.n_calls && A.xcall_prefetch) {
      if (closed) {
        if (active) e_next = e_call + A.call_elems;   // gpsisr keeps prn and stream
      } else {
        const gnsscorr_nco_cmd& nc = A.cmds[(int64_t)(k + 1) * A.cmd_step + chn];
        if (nc.prn > 0 && nc.prn <= 32)
          e_next = (int64_t)nc.stream * A.stream_stride * 2 + (int64_t)(k + 1) * A.call_elems;
      }
    }
    // keep one piece in flight: the rest of this call, then the next call's
    auto top_up = [&]() {
      while (iss == con) {
        int nk = q_k, np = q_p + 1;
        if (np >= n_pieces) {
          nk++;
          np = 0;
        }
        if (nk == k) issue(k, np, e_call);
        else if (nk == k + 1 && e_next >= 0) issue(k + 1, np, e_next);
        else break;
      }
    };
    if (active) top_up();

    Acc acc;
#pragma unroll
    for (int q = 0; q < 6; q++) acc.a[q] = 0;
    int e = -1;   // epoch of acc (-1: nothing yet)
    Seg g;
    // the carrier and code NCO phases at the lane's first sample, advanced by one
    // piece (kPieceSpan samples: uniform steps) per piece with full-rate adds, not
    // a 32 x 32-bit and a 64-bit multiply per piece (quarter rate)
    // (the carrier phase steps in g.p0 itself where the pair loops do not advance
    // it, i.e. with the LO words read ahead)
    const uint32_t p0_step = (uint32_t)kPieceSpan * c.cinc;
    if constexpr (kPF) g.p0 = c.P0 + (uint32_t)(lane * kPieceLen) * c.cinc - p0_step;
    uint64_t x_cur = (uint64_t)c.K0 + (uint64_t)(uint32_t)(lane * kPieceLen) * c.kinc2;
    const uint64_t x_step = (uint64_t)kPieceSpan * c.kinc2;
    for (int p = 0; active && p < n_pieces; p++) {
      const int n0 = p * kPieceSpan + lane * kPieceLen;
      const int L = max(0, min(kPieceLen, nsamp - n0));
      if constexpr (kPF) g.p0 += p0_step;   // c.P0 + n0 cinc
      else g.p0 = c.P0 + (uint32_t)n0 * c.cinc;
      // the piece's 16 LO word pairs (pair q: carrier phases p0 + 2q cinc and
      // p0 + (2q + 1) cinc, correlator.c:203-204), read before the piece's IF
      // wait so that both LDS round trips overlap
      uint32_t lwx[kPieceLen / 2], lwy[kPieceLen / 2];
      if (kPF && fast) {
        uint32_t pa = g.p0;
#pragma unroll
        for (int q = 0; q < kPieceLen / 2; q++) {
          const uint32_t pb = pa + c.cinc;
          const uint32_t off = ((pa >> 27) & 0x1Cu) | ((pb >> 24) & 0xE0u);   // 4 (a | b << 3)
          const uint8_t* t = reinterpret_cast<const uint8_t*>(s_lot) + off;
          lwx[q] = *reinterpret_cast<const uint32_t*>(t);
          lwy[q] = *reinterpret_cast<const uint32_t*>(t + 256);
          pa = pb + c.cinc;
        }
      }
      // ---- this lane's 32 samples as 16 pair words (4 chunks of 4)
      uint4 ch4[4];
      if constexpr (PK) {
        if constexpr (kX2) {
          auto x2 = [&](uint32_t w) {
            return make_uint4(s_x2[w & 0xFFu], s_x2[(w >> 8) & 0xFFu], s_x2[(w >> 16) & 0xFFu],
                              s_x2[w >> 24]);
          };
          ch4[0] = x2(pq0.x);
          ch4[1] = x2(pq0.y);
          ch4[2] = x2(pq1.x);
          ch4[3] = x2(pq1.y);
        } else {
          ch4[0] = if2_expand_word(pq0.x);
          ch4[1] = if2_expand_word(pq0.y);
          ch4[2] = if2_expand_word(pq1.x);
          ch4[3] = if2_expand_word(pq1.y);
        }
      } else {
        if (p * kPieceSpan + kPieceSpan > nsamp && (nsamp & 7)) {
          // the call's partial last chunk (nsamp not a multiple of 8; single
          // calls only): whole words and the odd sample by ordinary loads
          const int n_piece = p * kPieceSpan;
          const int valid = nsamp - n_piece;
          const int i = valid / 8;
          if (lane == (i & 63)) {
            const int rem = valid - i * 8;
            const uint32_t* g32 =
                reinterpret_cast<const uint32_t*>(A.ifbuf + e_call + 2 * (int64_t)n_piece) + 4 * i;
            uint32_t t[4] = {0u, 0u, 0u, 0u};
            for (int q = 0; q < rem / 2; q++) t[q] = g32[q];
            if (rem & 1) t[rem / 2] = (uint32_t)reinterpret_cast<const uint16_t*>(g32)[rem - 1];
            slot[slot_entry(i)] = make_uint4(t[0], t[1], t[2], t[3]);
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the piece has landed in the slot
        if (p == 0) STREAM_PSTAMP(2);
#pragma unroll
        for (int j = 0; j < 4; j++) ch4[j] = slot[slot_entry(4 * lane + j)];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ... and is in registers
      }
      con = __builtin_amdgcn_readfirstlane(con + 1);
      top_up();   // the slot just read takes the next piece
      const uint64_t X = x_cur;   // c.K0 + n0 kinc2
      x_cur += x_step;
      const uint64_t r0 = X >> 32;
      g.kph = (uint32_t)X;
      uint32_t ep = (uint32_t)e;   // (lanes past the call's end keep their epoch)
      if (L > 0) {
        if (fast) hc_after_fast(c, r0, invD, g.hc, g.ld, ep);
        else hc_after(c, r0, g.hc, g.ld, ep);
      }
      {   // a piece that starts in a later epoch than the lane's sums (rare; every
          // lane still active: flush_lanes' DPP scans)
        uint64_t any = __builtin_amdgcn_ballot_w64((int)ep != e);
        asm volatile("" : "+s"(any));
        if (any) {
          flush_lanes<true>((int)ep != e && e >= 0, acc, e, s_sum, lane);
          e = (int)ep;
        }
      }
      if (L == 0) continue;
      if (fast) {
        if constexpr (kPF) {
          g.cb = row[g.ld];
          g.nb = row[g.hc + 1];
          unpack8(g.cb, g.lb, g.pb, g.eb);
        } else {
          unpack8(row[g.ld], g.lb, g.pb, g.eb);
        }
        g.ti = g.tq = g.pi = g.pq = 0;
        g.carried = false;
        // intervals of kIv pairs: 3 (6 samples) whenever a half-chip lasts >= 6
        // samples; 4 (8 samples, 4 interval ends per piece instead of 6) when it
        // lasts >= 8, i.e. 8 kinc2 <= 2^32 (at 16.368 Msps: code rates up to the
        // nominal 2.046 MHz of half-chips), still at most one carry per interval
        auto full_piece = [&](auto dumps_tag, auto iv_tag) {
          constexpr bool kD = decltype(dumps_tag)::value;
          constexpr int kIv = decltype(iv_tag)::value;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t words[4] = {ch4[j].x, ch4[j].y, ch4[j].z, ch4[j].w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int q = 4 * j + i;
              if constexpr (kPF) pair2r<false>(words[i], lwx[q], lwy[q], c, g);
              else pair2s<false>(words[i], c, g, lox, loy);
              if (q % kIv == kIv - 1 || q == kPieceLen / 2 - 1)
                interval_end_s<kPF, kD>(c, g, acc, e, s_sum, row);
            }
          }
        };
        // a piece in which every lane's code carries fall at one offset j in each
        // of its four 8-sample intervals (chunk t = samples 8t .. 8t + 7, carry
        // between samples 8t + j - 1 and 8t + j): the part of a pair before the
        // carry has a mask fixed for the piece, so a pair is one AND and four dot4
        // (no NCO step or carry test per pair), and every interval ends on a carry
        auto aligned_piece = [&](const uint32_t (&mq)[4]) {
#pragma unroll
          for (int t = 0; t < 4; t++) {
            const uint32_t words[4] = {ch4[t].x, ch4[t].y, ch4[t].z, ch4[t].w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
              uint32_t lo_x, lo_y;
              if constexpr (kPF) {
                lo_x = lwx[4 * t + i];
                lo_y = lwy[4 * t + i];
              } else {
                const uint32_t p1 = g.p0 + c.cinc;
                const uint32_t idx = (g.p0 >> 29) | ((p1 >> 26) & 0x38u);
                lo_x = lox[idx];
                lo_y = loy[idx];
                g.p0 = p1 + c.cinc;
              }
              const uint32_t xm = words[i] & mq[i];
              g.ti = dot4(words[i], lo_x, g.ti);
              g.tq = dot4(words[i], lo_y, g.tq);
              g.pi = dot4(xm, lo_x, g.pi);
              g.pq = dot4(xm, lo_y, g.pq);
            }
            seg_flush(g.pi, g.pq, g.lb, g.pb, g.eb, acc);
            const int ri = g.ti - g.pi, rq = g.tq - g.pq;
            g.ti = g.pi = ri;
            g.tq = g.pq = rq;
            g.hc += 1u;   // no dump in the piece (the caller's ballot)
            if constexpr (kPF) {
              g.cb = g.nb;
              unpack8(g.cb, g.lb, g.pb, g.eb);
              g.nb = row[g.hc + 1];
            } else {
              g.ld = g.hc;
              unpack8(row[g.ld], g.lb, g.pb, g.eb);
            }
          }
        };
        if (__all(L == kPieceLen)) {
          // whether any lane's 32 samples hold a dump: its half-chip count at the
          // window start plus the window's code carries, (kph + 32 kinc2) >> 32,
          // reaches D (one dump per ~16 k samples, so 7 of 8 pieces have none and
          // skip the dump test at every interval end)
          const bool dump_here =
              g.hc + (uint32_t)(((uint64_t)g.kph + (uint64_t)kPieceLen * c.kinc2) >> 32) >= c.D;
          uint64_t anyd = __builtin_amdgcn_ballot_w64(dump_here);
          asm volatile("" : "+s"(anyd));
          using I3 = std::integral_constant<int, 3>;
          using I4 = std::integral_constant<int, 4>;
          bool aligned = false;
          if (TRACK_ALIGNED && TRACK_NODUMP_COPY && !anyd) {
            // j: samples before the lane's first carry (sample n has half-chip
            // hc + h(n), h(n) = (kph + n kinc2) >> 32), estimated in fp32 and
            // checked exactly.  h(j - 1) = 0, h(j) = 1, h(j + 23) = 3, h(j + 24) = 4
            // put the carries at j, j + 8, j + 16, j + 24: three spacings summing to
            // 24 from {floor P, ceil P} (P samples per half-chip) are all 8, and the
            // next carry (>= j + 31) is past the piece
            const float r = (4294967296.0f - (float)g.kph) * __builtin_amdgcn_rcpf((float)c.kinc2);
            const int j = min(8, max(1, (int)__builtin_ceilf(r)));
            // with Y = kph + j kinc2 and Z = Y + 24 kinc2: h(j) = 1 and h(j + 24) = 4 are
            // their high words; then h(j - 1) = 0 iff Y - kinc2 < 2^32, i.e. lo(Y) < kinc2,
            // and h(j + 23) = 3 iff lo(Z) < kinc2 (one 64-bit multiply, not four)
            const uint64_t Y = (uint64_t)g.kph + (uint64_t)(uint32_t)j * c.kinc2;
            const uint64_t Z = Y + 24ull * c.kinc2;
            const bool ok = (uint32_t)(Y >> 32) == 1u && (uint32_t)Y < c.kinc2 &&
                            (uint32_t)(Z >> 32) == 4u && (uint32_t)Z < c.kinc2;
            uint64_t bad = __builtin_amdgcn_ballot_w64(!ok);
            asm volatile("" : "+s"(bad));
            if (!bad) {
              uint32_t mq[4];
#pragma unroll
              for (int i = 0; i < 4; i++)
                mq[i] = j >= 2 * i + 2 ? 0xFFFFFFFFu : (j == 2 * i + 1 ? 0xFFFFu : 0u);
              aligned_piece(mq);
              aligned = true;
            }
          }
          if (aligned) {
          } else if (TRACK_NODUMP_COPY && !anyd) {
            if (TRACK_IV4 && c.kinc2 <= kIv4Kinc2) full_piece(std::false_type{}, I4{});
            else full_piece(std::false_type{}, I3{});
          } else {
            full_piece(std::true_type{}, I3{});
          }
        } else {
          const int np = L >> 1;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t words[4] = {ch4[j].x, ch4[j].y, ch4[j].z, ch4[j].w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const int q = 4 * j + i;
              if constexpr (kPF) {
                if (q < np) pair2r<false>(words[i], lwx[q], lwy[q], c, g);
                else if (q == np && (L & 1)) pair2r<true>(words[i] & 0xFFFFu, lwx[q], lwy[q], c, g);
              } else {
                if (q < np) pair2s<false>(words[i], c, g, lox, loy);
                else if (q == np && (L & 1)) pair2s<true>(words[i] & 0xFFFFu, c, g, lox, loy);
              }
              if (q % 3 == 2 || q == kPieceLen / 2 - 1) interval_end_s<kPF>(c, g, acc, e, s_sum, row);
            }
          }
        }
        seg_flush(g.ti, g.tq, g.lb, g.pb, g.eb, acc);   // the open segment
      } else {
        uint32_t hc = g.hc;
        int lb, pb, eb;
        if (pk_lds) {
          unpack8(row[g.ld], lb, pb, eb);
        } else {
          const uint32_t tw = A.pk[c.base + (int)g.ld];
          lb = (int)(int8_t)(tw & 0xFFu);
          pb = (int)(int8_t)((tw >> 8) & 0xFFu);
          eb = (int)(int8_t)((tw >> 16) & 0xFFu);
        }
        uint32_t phase = g.p0, kph = g.kph;
        auto per_sample = [&](auto row_tag) {
          constexpr bool kRow = decltype(row_tag)::value;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const uint32_t words[4] = {ch4[j].x, ch4[j].y, ch4[j].z, ch4[j].w};
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
              for (int hh = 0; hh < 2; hh++)
                if (2 * (4 * j + i) + hh < L)
                  corr_sample_s<kRow>(sbyte((int)words[i], 2 * hh),
                                      sbyte((int)words[i], 2 * hh + 1), phase, kph, c, hc, lb, pb,
                                      eb, acc, e, s_sum, row, A.pk);
          }
        };
        if (pk_lds) per_sample(std::true_type{});
        else per_sample(std::false_type{});
      }
    }
    flush_lanes<false>(e >= 0, acc, e, s_sum, lane);   // (the next call starts from zero)
    if (!active && iss != con) {
      // a prefetch for a call that turned out idle must land before the slot is reused
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      con = iss;
      q_k = q_p = -1;
    }
    wave_lds_sync();   // every lane's flushes land before lane 0 reads the sums
    STREAM_PSTAMP(3);
    // ---- the channel's epilogue (and closed loop: its gpsisr step) on lane 0; the
    // epoch sums are complete (the LDS operations of a wave execute in order)
    // lane 0's new state and command go to every lane by readfirstlane (an LDS
    // round trip would need a fence: without one the compiler may hoist the
    // other lanes' reads above lane 0's writes)
    uint32_t bw[20];
#pragma unroll
    for (int i = 0; i < 20; i++) bw[i] = 0u;
    if (lane == 0) {
      const uint64_t Rtot = ((uint64_t)c.K0 + (uint64_t)nsamp * c.kinc2) >> 32;
      gnsscorr_chan_state nst;
      const gnsscorr_track_result rr = channel_epilogue(
          c, cmd, st, chn, active, active ? n_dumps_after(c, Rtot) : 0u, Rtot, nsamp, tic_k,
          [&](int i) { return (uint32_t)s_sum[i]; }, A.res + (int64_t)k * C, A.state,
          A.n_calls == 1 ? A.all_dumps : nullptr, A.max_dumps, &nst);
      gnsscorr_nco_cmd r = cmd;
      if constexpr (CLOSED) {   // osgpsisr.c:360-768, osg_isr_kernel's body
        gnsscorr_osg_loop lc = A.loops[chn];
        osgisr::isr_step(A.lk, lc, r, rr);
        A.loops[chn] = lc;
        if (A.hist) A.hist[(int64_t)k * C + chn] = lc;
        if (k + 1 == A.n_calls) A.cmds[chn] = r;
      }
      memcpy(bw, &nst, sizeof nst);
      memcpy(bw + 14, &r, sizeof r);
    }
    {
      static_assert(sizeof(gnsscorr_chan_state) == 56 && sizeof(gnsscorr_nco_cmd) == 24, "bw");
      uint32_t* sv = reinterpret_cast<uint32_t*>(&st);
#pragma unroll
      for (int i = 0; i < 14; i++) sv[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)bw[i]);
      if (closed) {
        uint32_t* rv = reinterpret_cast<uint32_t*>(&cmd);
#pragma unroll
        for (int i = 0; i < 6; i++) rv[i] = (uint32_t)__builtin_amdgcn_readfirstlane((int)bw[14 + i]);
      }
    }
  }
  STREAM_PSTAMP(5);
}

}  // namespace

// ============================================================================
// context / C ABI
// ============================================================================
struct gnsscorr_track_ctx {
  gnsscorr_track_cfg cfg;
  hipStream_t stream = nullptr;
  uint32_t* d_pk = nullptr;
  uint8_t* d_pk8 = nullptr;   // the same table as 2-bit E/P/L fields (unpack8)
  gnsscorr_chan_state* d_state = nullptr;
  gnsscorr_nco_cmd* d_cmds = nullptr;
  gnsscorr_track_result* d_res = nullptr;
  int32_t* d_dumps = nullptr;
  int8_t* d_if = nullptr;
  size_t if_cap = 0;
  int max_dumps = 0;
  int64_t tic = 0, tic_ref = 0;
  int stage_if = 1;   // GNSSCORR_TRACK_STAGE_IF=0: lanes read their IF runs from global memory
  int cpw_override = 0;   // GNSSCORR_TRACK_CPW: channels per workgroup
  int pieces_all = 0;     // GNSSCORR_TRACK_PIECES=1: the piece path for receivers too (A/B)
  int stream_kernel = 1;  // GNSSCORR_TRACK_STREAM=0: IQ calls on the per-call workgroup
                          // kernel instead of osg_stream_kernel (A/B)
  int balance = 1;         // GNSSCORR_TRACK_BALANCE=0: no LDS padding for an even spread (A/B)
  int xcall_prefetch = 1;  // GNSSCORR_TRACK_XPF=0: no cross-call piece prefetch (A/B)
  int n_cu = 256;
  size_t lds_max = 0;     // LDS bytes a workgroup may allocate (gnsscorr_device_lds_bytes)
};

extern "C" int gnsscorr_track_iq(const gnsscorr_track_ctx* ctx) { return ctx && (ctx->cfg.iq & GNSSCORR_IF_IQ); }
static bool packed(const gnsscorr_track_ctx* c) { return (c->cfg.iq & GNSSCORR_IF_PACKED2) != 0; }
static int bps_of(const gnsscorr_track_ctx* c) { return (c->cfg.iq & GNSSCORR_IF_IQ) ? 2 : 1; }
// bytes of `samples` consecutive samples of one stream in the context's format
extern "C" int64_t gnsscorr_track_if_bytes(const gnsscorr_track_ctx* c, int64_t samples) {
  return if_bytes(samples * bps_of(c), packed(c));
}

static int set_dev(int dev) {
  HIP_TRY(hipSetDevice(dev));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_create(gnsscorr_track_ctx** out, const gnsscorr_track_cfg* cfg) {
  if (!out || !cfg || cfg->n_channels < 1 || cfg->max_nsamp < 1 || cfg->max_nsamp > kMaxNsamp ||
      (cfg->iq & ~(GNSSCORR_IF_IQ | GNSSCORR_IF_PACKED2))) {
    gnsscorr_set_error("gnsscorr_track_create: bad config (n_channels>=1, 1<=max_nsamp<=%d, "
                       "iq = GNSSCORR_IF_* flags)", kMaxNsamp);
    return GNSSCORR_EINVAL;
  }
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gnsscorr_set_error("gnsscorr_track_create: no HIP device");
    return GNSSCORR_ENODEV;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    gnsscorr_set_error("gnsscorr_track_create: device %d out of range", cfg->device);
    return GNSSCORR_EINVAL;
  }
  int rc = set_dev(cfg->device);
  if (rc) return rc;
  auto* c = new gnsscorr_track_ctx();
  c->cfg = *cfg;
  c->lds_max = (size_t)gnsscorr_device_lds_bytes(cfg->device);
  c->max_dumps = cfg->max_nsamp / GNSSCORR_OSG_ROW + 2;
  c->tic_ref = (int64_t)(cfg->samp_rate * cfg->tic_period);
  c->tic = c->tic_ref;
  if (const char* e = getenv("GNSSCORR_TRACK_STAGE_IF")) c->stage_if = atoi(e) != 0;
  if (const char* e = getenv("GNSSCORR_TRACK_CPW")) c->cpw_override = atoi(e);
  if (const char* e = getenv("GNSSCORR_TRACK_PIECES")) c->pieces_all = atoi(e) != 0;
  if (const char* e = getenv("GNSSCORR_TRACK_STREAM")) c->stream_kernel = atoi(e) != 0;
  if (const char* e = getenv("GNSSCORR_TRACK_BALANCE")) c->balance = atoi(e) != 0;
  if (const char* e = getenv("GNSSCORR_TRACK_XPF")) c->xcall_prefetch = atoi(e) != 0;
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, cfg->device) !=
          hipSuccess || c->n_cu < 1)
    c->n_cu = 256;

  const int C = cfg->n_channels;
  auto fail = [&](int code) {
    gnsscorr_track_destroy(c);
    return code;
  };
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc(&c->d_pk, sizeof(uint32_t) * GNSSCORR_OSG_PK_LEN) != hipSuccess ||
      hipMalloc(&c->d_pk8, GNSSCORR_OSG_PK_LEN + 64) != hipSuccess ||   // +64: whole-dword row staging
      hipMalloc(&c->d_state, sizeof(gnsscorr_chan_state) * C) != hipSuccess ||
      hipMalloc(&c->d_cmds, sizeof(gnsscorr_nco_cmd) * C) != hipSuccess ||
      hipMalloc(&c->d_res, sizeof(gnsscorr_track_result) * C) != hipSuccess ||
      hipMalloc(&c->d_dumps, sizeof(int32_t) * 6 * (size_t)C * c->max_dumps) != hipSuccess) {
    gnsscorr_set_error("gnsscorr_track_create: device allocation failed");
    return fail(GNSSCORR_ENOMEM);
  }
  uint32_t* pk = (uint32_t*)malloc(sizeof(uint32_t) * GNSSCORR_OSG_PK_LEN);
  if (!pk) return fail(GNSSCORR_ENOMEM);
  gnsscorr_osg_packed_table(pk);
  hipError_t e = hipMemcpy(c->d_pk, pk, sizeof(uint32_t) * GNSSCORR_OSG_PK_LEN, hipMemcpyHostToDevice);
  // pack8: each int8 bit (-1 / 0 / +1) of {late, prompt, early} as a 2-bit field
  for (int i = 0; i < GNSSCORR_OSG_PK_LEN; i++) {
    uint32_t b = 0;
    for (int k = 0; k < 3; k++) b |= ((uint32_t)(int8_t)(pk[i] >> (8 * k)) & 3u) << (2 * k);
    reinterpret_cast<uint8_t*>(pk)[i] = (uint8_t)b;
  }
  if (e == hipSuccess) e = hipMemset(c->d_pk8, 0, GNSSCORR_OSG_PK_LEN + 64);
  if (e == hipSuccess) e = hipMemcpy(c->d_pk8, pk, GNSSCORR_OSG_PK_LEN, hipMemcpyHostToDevice);
  free(pk);
  if (e != hipSuccess || hipMemset(c->d_state, 0, sizeof(gnsscorr_chan_state) * C) != hipSuccess) {
    gnsscorr_set_error("gnsscorr_track_create: upload failed: %s", hipGetErrorString(e));
    return fail(GNSSCORR_EDEVICE);
  }
  *out = c;
  return GNSSCORR_OK;
}

// Layout hint (round 2: per-channel LDS staging for one stream per channel).
// Since round 3 every workgroup picks its IF path itself -- the shared LDS
// stage when its channels read one stream, the per-wave piece path otherwise --
// so the hint is accepted and has no effect.
extern "C" int gnsscorr_track_set_layout(gnsscorr_track_ctx* c, int one_stream_per_channel) {
  if (!c || one_stream_per_channel < 0 || one_stream_per_channel > 1) {
    gnsscorr_set_error("gnsscorr_track_set_layout: bad arguments");
    return GNSSCORR_EINVAL;
  }
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_destroy(gnsscorr_track_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  void* bufs[] = {c->d_pk, c->d_pk8, c->d_state, c->d_cmds, c->d_res, c->d_dumps, c->d_if};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_max_dumps(const gnsscorr_track_ctx* c) { return c ? c->max_dumps : 0; }

extern "C" int64_t gnsscorr_track_next_tic(gnsscorr_track_ctx* c, int64_t nsamp) {
  // correlator.c:155-165
  if (c->tic < nsamp) {
    const int64_t t = c->tic;
    c->tic += c->tic_ref - nsamp;
    return t;
  }
  c->tic -= nsamp;
  return -1;
}

// osg_stream_kernel: n_calls consecutive calls of every channel in one launch
// (call k reads the IF at + k * nsamp samples of each stream and the commands
// at d_cmds + k * cmd_step; the results go to d_res + k * n_channels).  tic: the
// first call's TIC sample (tic_explicit) or the TIC counter to step per call.
// lcfg/d_loops: the closed loop, every channel's gpsisr step after each call.
// Returns GNSSCORR_TRACK_NOT_FUSED when the kernel does not serve the context
// or the shape (I-only streams, LDS, alignment of later calls).
static int launch_stream(gnsscorr_track_ctx* c, const int8_t* d_if, int64_t stride, int64_t nsamp,
                         int n_calls, gnsscorr_nco_cmd* d_cmds, int cmd_step,
                         gnsscorr_track_result* d_res, int32_t* d_dumps, int64_t tic,
                         int tic_explicit, const gnsscorr_osg_loop_cfg* lcfg,
                         gnsscorr_osg_loop* d_loops, gnsscorr_osg_loop* d_hist) {
  const bool pk = packed(c), iq = bps_of(c) == 2;
  if (!iq || !c->stream_kernel) return GNSSCORR_TRACK_NOT_FUSED;
  if (nsamp < 1 || nsamp > c->cfg.max_nsamp) {
    gnsscorr_set_error("nsamp %lld outside [1, max_nsamp=%d]", (long long)nsamp, c->cfg.max_nsamp);
    return GNSSCORR_EINVAL;
  }
  if (((uintptr_t)d_if & (pk ? 7 : 15)) || ((stride * 2) & (pk ? 31 : 15))) {
    gnsscorr_set_error("IF base and stream stride must be %d-byte aligned", pk ? 8 : 16);
    return GNSSCORR_EINVAL;
  }
  // later calls start at + k * nsamp samples: the same alignment, and whole
  // 8-sample chunks (the partial-chunk path is for single calls)
  if (n_calls > 1 && ((nsamp * 2) & (pk ? 31 : 15))) return GNSSCORR_TRACK_NOT_FUSED;
  const int C = c->cfg.n_channels;
  size_t dyn = (size_t)stream_wave_lds(pk, (int)nsamp) * kStreamCh;
  constexpr size_t kStatic = 2048;   // s_lot, s_x2 (packed), with margin
  if (dyn + kStatic > c->lds_max) return GNSSCORR_TRACK_NOT_FUSED;
  // A launch takes as long as its busiest CU.  The dispatcher fills a CU with
  // as many workgroups as its resources allow, so at 768 workgroups on 256 CUs
  // some CUs got 4-5 while others got 2 (wave stamps: pieces p10 16.6 / p90
  // 27 us).  Asking for enough LDS that at most ceil(workgroups / CUs) fit on
  // a CU spreads them evenly.
  const int n_wg = (C + kStreamCh - 1) / kStreamCh;
  const int per_cu = (n_wg + c->n_cu - 1) / c->n_cu;
  // Only when the launch has more workgroups than CUs: with at most one per CU
  // the dispatcher spreads them already, and the padding would only lock other
  // streams' kernels out of those CUs' LDS (co-residency).
  if (c->balance && n_wg > c->n_cu) {
    const size_t cap = c->lds_max / (size_t)(per_cu + 1) + 16;   // per_cu + 1 no longer fit
    if (cap > dyn && (cap + kStatic) * per_cu <= c->lds_max) dyn = cap;
  }
  StreamArgs A;
  memset(&A, 0, sizeof A);
  A.ifbuf = d_if;
  A.stream_stride = stride;
  A.call_elems = nsamp * 2;
  A.nsamp = (int)nsamp;
  A.n_channels = C;
  A.n_calls = n_calls;
  A.cmd_step = cmd_step;
  A.cmds = d_cmds;
  A.state = c->d_state;
  A.res = d_res;
  A.all_dumps = d_dumps;
  A.max_dumps = c->max_dumps;
  A.pk = c->d_pk;
  A.pk8 = c->d_pk8;
  A.tic = tic;
  A.tic_ref = c->tic_ref;
  A.tic_explicit = tic_explicit;
  A.xcall_prefetch = c->xcall_prefetch;
  if (lcfg) A.lk = *lcfg;
  A.loops = d_loops;
  A.hist = d_hist;
  dim3 grid(n_wg), block(64 * kStreamCh);
  // the closed loop's gpsisr in its own instantiation: its registers stay out of
  // the open-loop kernel
  if (pk && d_loops) hipLaunchKernelGGL((osg_stream_kernel<true, true>), grid, block, dyn, c->stream, A);
  else if (pk) hipLaunchKernelGGL((osg_stream_kernel<true, false>), grid, block, dyn, c->stream, A);
  else if (d_loops) hipLaunchKernelGGL((osg_stream_kernel<false, true>), grid, block, dyn, c->stream, A);
  else hipLaunchKernelGGL((osg_stream_kernel<false, false>), grid, block, dyn, c->stream, A);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

static int launch(gnsscorr_track_ctx* c, const int8_t* d_if, int64_t stride, int64_t nsamp,
                  const gnsscorr_nco_cmd* d_cmds, gnsscorr_track_result* d_res,
                  int32_t* d_dumps, int64_t tic_count) {
  if (nsamp < 1 || nsamp > c->cfg.max_nsamp) {
    gnsscorr_set_error("nsamp %lld outside [1, max_nsamp=%d]", (long long)nsamp, c->cfg.max_nsamp);
    return GNSSCORR_EINVAL;
  }
  const int bps = bps_of(c);
  const bool pk = packed(c), iq = bps == 2;
  // 16-byte aligned int8 runs; packed runs are read in 8-byte words
  if (((uintptr_t)d_if & (pk ? 7 : 15)) || ((stride * bps) & (pk ? 31 : 15))) {
    gnsscorr_set_error("IF base and stream stride must be %d-byte aligned", pk ? 8 : 16);
    return GNSSCORR_EINVAL;
  }
  const int C = c->cfg.n_channels;
  if (iq && c->stream_kernel) {
    const int rs = launch_stream(c, d_if, stride, nsamp, 1, const_cast<gnsscorr_nco_cmd*>(d_cmds),
                                 0, d_res, d_dumps, tic_count, 1, nullptr, nullptr, nullptr);
    if (rs != GNSSCORR_TRACK_NOT_FUSED) return rs;
  }
  int threads = (int)((nsamp + kRun - 1) / kRun);
  threads = (threads + 63) & ~63;
  const size_t stage_bytes = (size_t)((nsamp + kRun - 1) / kRun) * kPitch * 16;
  int stage = iq && c->stage_if && stage_bytes <= (size_t)kStageMaxBytes;
  if (stage && c->pieces_all) stage = 4;
  // dynamic LDS: epoch sums, E/P/L row bytes, then one region that holds either
  // the workgroup's shared IF stage or the waves' 4 KiB piece slots
  auto lds_bytes = [&](int cpw) {
    const size_t sum_bytes = (size_t)((cpw * ((int)nsamp / GNSSCORR_OSG_ROW + 2) * 6 + 3) & ~3) * 4;
    const size_t slots = (size_t)(threads / 64) * cpw * kStage2Bytes;
    return sum_bytes + (iq ? (size_t)cpw * kPk8Stage +
                                 (stage ? (stage_bytes > slots ? stage_bytes : slots) : 0) : 0);
  };
  // Channels per workgroup: as many as fit 1024 threads (they share one staged
  // IF copy).  The 1.5-round tail at 3072 channels (768 workgroups, 512
  // resident) is cheaper than smaller workgroups (MI355X, 3072 x 1 ms:
  // cpw 4 33.4 us, 3 35.2, 2 34.1, 1 46.4); GNSSCORR_TRACK_CPW overrides.
  int cpw = 1;
  auto pick_cpw = [&]() {
    cpw = min(kMaxCpw, kMaxThreads / threads);
    if (c->cpw_override > 0) cpw = min(cpw, c->cpw_override);
    // the LDS must fit beside the static LDS (s_lo, s_stream, s_short: < 1 KiB)
    while (cpw > 1 && lds_bytes(cpw) + 1024 > c->lds_max) cpw--;
  };
  pick_cpw();
  if (stage && lds_bytes(cpw) + 1024 > c->lds_max) {   // no room for the IF stage or
    stage = 0;                                          // the piece slots: lane reads
    pick_cpw();
  }
  if (lds_bytes(cpw) + 1024 > c->lds_max) {
    gnsscorr_set_error("gnsscorr_track: nsamp %lld needs %zu B of LDS per workgroup, the device "
                       "allows %zu", (long long)nsamp, lds_bytes(cpw) + 1024, c->lds_max);
    return GNSSCORR_EINVAL;
  }
  dim3 grid((C + cpw - 1) / cpw), block(threads * cpw);
  const size_t dyn = lds_bytes(cpw);
#define TRACK_LAUNCH(IQ, PK, ST)                                                               \
  hipLaunchKernelGGL((osg_track_kernel<IQ, PK>), grid, block, dyn, c->stream, d_if, stride,    \
                     (int)nsamp, C, cpw, d_cmds, c->d_state, d_res, d_dumps, c->max_dumps,     \
                     c->d_pk, c->d_pk8, tic_count, ST)
  if (iq && pk)
    TRACK_LAUNCH(true, true, stage);
  else if (iq)
    TRACK_LAUNCH(true, false, stage);
  else if (pk)
    TRACK_LAUNCH(false, true, 0);
  else
    TRACK_LAUNCH(false, false, 0);
#undef TRACK_LAUNCH
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track(gnsscorr_track_ctx* c, const int8_t* h_if, int64_t stride,
                              int n_streams, int64_t nsamp, const gnsscorr_nco_cmd* h_cmds,
                              gnsscorr_track_result* h_res, int32_t* h_all_dumps, int* tic_fired) {
  if (!c || !h_if || !h_cmds || !h_res || n_streams < 1 || nsamp < 1) {
    gnsscorr_set_error("gnsscorr_track: bad arguments");
    return GNSSCORR_EINVAL;
  }
  const int C = c->cfg.n_channels;
  for (int i = 0; i < C; i++) {
    if (h_cmds[i].prn < 0 || h_cmds[i].prn > 32 || h_cmds[i].stream < 0 ||
        h_cmds[i].stream >= n_streams) {
      gnsscorr_set_error("gnsscorr_track: channel %d: prn %d / stream %d invalid", i,
                         h_cmds[i].prn, h_cmds[i].stream);
      return GNSSCORR_EINVAL;
    }
  }
  if (n_streams == 1) stride = 0;
  if (n_streams > 1 && stride < nsamp) {
    gnsscorr_set_error("gnsscorr_track: stream_stride < nsamp");
    return GNSSCORR_EINVAL;
  }
  int rc = set_dev(c->cfg.device);
  if (rc) return rc;
  const int bps = bps_of(c);
  const bool pk = packed(c);
  if (pk && n_streams > 1 && (stride * bps) & 3) {
    gnsscorr_set_error("gnsscorr_track: packed streams need a whole-byte stream stride");
    return GNSSCORR_EINVAL;
  }
  // device copy with an aligned stride (16 int8 bytes / 8 packed bytes = 32 elements)
  const int64_t al = pk ? 32 : 16;
  const int64_t dstride = n_streams > 1 ? ((stride * bps + al - 1) & ~(al - 1)) / bps : 0;
  const size_t need = (size_t)if_bytes((n_streams - 1) * dstride * bps + ((nsamp * bps + al - 1) & ~(al - 1)), pk);
  if (need > c->if_cap) {
    if (c->d_if) (void)hipFree(c->d_if);
    c->d_if = nullptr;
    c->if_cap = 0;
    HIP_TRY(hipMalloc(&c->d_if, need));
    c->if_cap = need;
  }
  if (n_streams == 1 || dstride == stride) {
    HIP_TRY(hipMemcpyAsync(c->d_if, h_if, (size_t)if_bytes(((n_streams - 1) * stride + nsamp) * bps, pk),
                           hipMemcpyHostToDevice, c->stream));
  } else {
    HIP_TRY(hipMemcpy2DAsync(c->d_if, if_bytes(dstride * bps, pk), h_if, if_bytes(stride * bps, pk),
                             if_bytes(nsamp * bps, pk), n_streams, hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(hipMemcpyAsync(c->d_cmds, h_cmds, sizeof(gnsscorr_nco_cmd) * C, hipMemcpyHostToDevice,
                         c->stream));
  const int64_t tic = gnsscorr_track_next_tic(c, nsamp);
  rc = launch(c, c->d_if, dstride, nsamp, c->d_cmds, c->d_res, h_all_dumps ? c->d_dumps : nullptr,
              tic);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(h_res, c->d_res, sizeof(gnsscorr_track_result) * C,
                         hipMemcpyDeviceToHost, c->stream));
  if (h_all_dumps)
    HIP_TRY(hipMemcpyAsync(h_all_dumps, c->d_dumps, sizeof(int32_t) * 6 * (size_t)C * c->max_dumps,
                           hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (tic_fired) *tic_fired = tic >= 0;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_dev(gnsscorr_track_ctx* c, const int8_t* d_if, int64_t stride,
                                  int64_t nsamp, const gnsscorr_nco_cmd* d_cmds,
                                  gnsscorr_track_result* d_res, int32_t* d_all_dumps,
                                  int64_t tic_count) {
  if (!c || !d_if || !d_cmds || !d_res) {
    gnsscorr_set_error("gnsscorr_track_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  int rc = set_dev(c->cfg.device);
  if (rc) return rc;
  return launch(c, d_if, stride, nsamp, d_cmds, d_res, d_all_dumps, tic_count);
}

extern "C" int gnsscorr_track_dev_isr(gnsscorr_track_ctx* c, const int8_t* d_if, int64_t stride,
                                      int64_t nsamp, int n_calls, gnsscorr_nco_cmd* d_cmds,
                                      gnsscorr_track_result* d_res, int n_loops,
                                      const gnsscorr_osg_loop_cfg* cfg, gnsscorr_osg_loop* d_loops,
                                      gnsscorr_osg_loop* d_hist) {
  if (!c || !d_if || !d_cmds || !d_res || !cfg || !d_loops || n_calls < 1) {
    gnsscorr_set_error("gnsscorr_track_dev_isr: bad arguments");
    return GNSSCORR_EINVAL;
  }
  if (n_loops != c->cfg.n_channels) return GNSSCORR_TRACK_NOT_FUSED;
  int rc = set_dev(c->cfg.device);
  if (rc) return rc;
  rc = launch_stream(c, d_if, stride, nsamp, n_calls, d_cmds, 0, d_res, nullptr, c->tic, 0, cfg,
                     d_loops, d_hist);
  if (rc == GNSSCORR_OK)   // the kernel stepped the TIC counter once per call; so does the host
    for (int k = 0; k < n_calls; k++) (void)gnsscorr_track_next_tic(c, nsamp);
  return rc;
}

extern "C" int gnsscorr_track_replay_dev(gnsscorr_track_ctx* c, const int8_t* d_if, int64_t stride,
                                         int64_t nsamp, int n_steps,
                                         const gnsscorr_nco_cmd* d_cmds,
                                         gnsscorr_track_result* d_res) {
  if (!c || !d_if || !d_cmds || !d_res || n_steps < 1) {
    gnsscorr_set_error("gnsscorr_track_replay_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  int rc = set_dev(c->cfg.device);
  if (rc) return rc;
  const int C = c->cfg.n_channels;
  // every call in one osg_stream_kernel launch where it serves the context
  rc = launch_stream(c, d_if, stride, nsamp, n_steps, const_cast<gnsscorr_nco_cmd*>(d_cmds), C,
                     d_res, nullptr, c->tic, 0, nullptr, nullptr, nullptr);
  if (rc == GNSSCORR_OK) {
    for (int k = 0; k < n_steps; k++) (void)gnsscorr_track_next_tic(c, nsamp);
    return GNSSCORR_OK;
  }
  if (rc != GNSSCORR_TRACK_NOT_FUSED) return rc;
  for (int k = 0; k < n_steps; k++) {
    const int64_t tic = gnsscorr_track_next_tic(c, nsamp);
    rc = launch(c, d_if + gnsscorr_track_if_bytes(c, (int64_t)k * nsamp), stride, nsamp,
                d_cmds + (int64_t)k * C,
                d_res + (int64_t)k * C, nullptr, tic);
    if (rc) return rc;
  }
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_get_state(gnsscorr_track_ctx* c, gnsscorr_chan_state* h) {
  if (!c || !h) return GNSSCORR_EINVAL;
  int rc = set_dev(c->cfg.device);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(h, c->d_state, sizeof(gnsscorr_chan_state) * c->cfg.n_channels,
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_set_state(gnsscorr_track_ctx* c, const gnsscorr_chan_state* h) {
  if (!c || !h) return GNSSCORR_EINVAL;
  int rc = set_dev(c->cfg.device);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(c->d_state, h, sizeof(gnsscorr_chan_state) * c->cfg.n_channels,
                         hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_track_sync(gnsscorr_track_ctx* c) {
  if (!c) return GNSSCORR_EINVAL;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" void* gnsscorr_track_stream(gnsscorr_track_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int gnsscorr_device_lds_bytes(int device) {
  int blk = 0, cu = 0;
  if (hipDeviceGetAttribute(&blk, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess)
    blk = 0;
  // gfx950 lets one workgroup allocate the CU's whole 160 KiB LDS, while the
  // runtime's per-block attribute may report the older 64 KiB; elsewhere the
  // per-block attribute is the limit
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess &&
      strncmp(prop.gcnArchName, "gfx950", 6) == 0 &&
      hipDeviceGetAttribute(&cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device) ==
          hipSuccess && cu > blk)
    return cu;
  return blk;
}

extern "C" int gnsscorr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
