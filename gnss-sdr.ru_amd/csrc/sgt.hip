// sgt.hip -- SoftGNSS float tracking loop ("sgt") on gfx950.
//
// The Scilab receivers track one channel at a time over a recorded file
// (GLONASS/L1/tracking.sci:150-400, GPS/L1/tracking.sci:124-360).  Here the
// whole record lives in HBM and one workgroup runs one channel's loop for
// many epochs without leaving the GPU:
//
//  epoch (uniform scalars, every thread computes the same fp64 values):
//    step    = codeFreq / fs                             tracking.sci:248
//    blksize = ceil((L - remCode) / step)                tracking.sci:250
//  samples (k = tid + j*T, coalesced int8 I,Q loads):
//    code index  ceil((remCode -/+ spc) + k*step)  -> padded [c(end) c c(1)]
//                (:282-299, fp64 with contraction off: bit-exact indices)
//    carrier     exp(i*((2*pi*f)*(k/fs) + remCarr)): one fp64 sincos per
//                thread, then an fp64 rotation per T samples (:305-313)
//    sums        I = code*imag(carr*raw), Q = code*real(carr*raw) (:316-326),
//                code +-1 applied as an fp64 sign flip (table of sign masks)
//  chunked path (default when 15*step < 1): kC consecutive samples per lane
//    and chunk, exact index of the chunk's first sample plus the exact
//    crossing to the next chip, code by position, carrier as an LDS table
//    W_n times one rotation per chunk (run_chunks below)
//  reduction: wavefront xor-shuffles, per-wave partials in LDS (double
//    buffered by epoch parity -> one barrier per epoch), every thread adds the
//    wave partials in the same order and runs the loop filters itself, so the
//    state stays uniform without a broadcast.
//  loop (closed_loop=1): FLL-assisted PLL + DLL, tracking.sci:329-375.
//
// Roofline: fp64 VALU (~27 DP ops per sample); HBM is 2 B/sample.
#include <hip/hip_runtime.h>
#include <type_traits>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "gnsscorr_internal.h"

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      gnsscorr_set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                         __LINE__);                                                     \
      return GNSSCORR_EDEVICE;                                                          \
    }                                                                                   \
  } while (0)

namespace {

constexpr int kMaxCode = 1023;
constexpr int kPadLen = kMaxCode + 2;
constexpr int kMaxWaves = 16;
#ifndef SGT_KC32
#define SGT_KC32 1
#endif
#ifndef SGT_WPE
#define SGT_WPE 3
#endif
#ifndef SGT_PREFIX
#define SGT_PREFIX 1
#endif
// chunked path, SGT_PREFIX: per-lane prefix sums of W_n*raw over sub-blocks of
// kSub samples staged in LDS (kSub x 64 x 16 B per wave), read back at each
// arm's crossing, instead of a code select and two FMAs per arm and sample
#ifndef SGT_KSUB
#define SGT_KSUB 16
#endif
// wave mode: chip-aligned chunks (run_chips) instead of the prefix columns,
// which then stay out of the wave kernel's LDS
#ifndef SGT_CHIPS
#define SGT_CHIPS 1
#endif
#ifndef SGT_CHIP_GROUP
#define SGT_CHIP_GROUP 4
#endif
#ifndef SGT_CHIP_FMA
#define SGT_CHIP_FMA 1
#endif
#ifndef SGT_CHIP_PF
#define SGT_CHIP_PF 1     // the next chunk's IF words loaded during this chunk
#endif
constexpr int kSub = SGT_KSUB;
constexpr int kPfWaveBytes = kSub * 64 * 16;
__host__ __device__ constexpr bool sgt_prefix(int maxt) {
  return SGT_PREFIX && maxt <= 256 && !(SGT_CHIPS && maxt == 64);
}
__host__ __device__ constexpr size_t sgt_tab_bytes(int code_length) {
  return ((size_t)(code_length + 3) * sizeof(double) + 15) & ~(size_t)15;   // s_sgn + guard
}

struct SgtParams {
  int system, file_type, switch_iq, code_length, chunked;
  int code_nco_variant, abs_sample_variant;   // tracking.sci:366/367, :379/:384
  double fs, code_basis, if_freq, l1_if_step, glo_zero, spc;
  double tau1, tau2, k1, k2, k3, pdi_code;
};

// End of one epoch of blk samples whose six sums are S (I_E, I_P, I_L, Q_E,
// Q_P, Q_L): the carry-over (tracking.sci:301-313), and closed loop the
// FLL-assisted PLL (:329-351) and the DLL (:353-375), then the record
// (:377-398).  One definition for the tracking kernel and the sums-replay
// kernel, so the replay against the reference's recorded run
// (tests/test_sgt_trackres_gpu.py) checks the code the tracker runs.
template <bool CLOSED>
__device__ __forceinline__ gnsscorr_sgt_epoch sgt_epoch_end(const SgtParams& p,
                                                            gnsscorr_sgt_chan& c, int blk,
                                                            double step, const double (&S)[6]) {
#pragma clang fp contract(off)
  const double I_E = S[0], I_P = S[1], I_L = S[2], Q_E = S[3], Q_P = S[4], Q_L = S[5];
  const double dL = (double)p.code_length, twopi = 2.0 * M_PI;
  const double A = (c.carr_freq * 2.0) * M_PI;        // (carrFreq * 2.0 * %pi)
  // carry-over (tracking.sci:301-313)
  const double tlast = c.rem_code + (double)(blk - 1) * step;   // tcode(blksize), prompt range
  c.rem_code = (tlast + step) - dL;
  const double last = A * ((double)blk / p.fs) + c.rem_carr;
  c.rem_carr = last - trunc(last / twopi) * twopi;
  c.pos += blk;
  double code_err = 0, carr_err = 0;
  if (CLOSED) {
    // FLL-assisted PLL (tracking.sci:329-353)
    const double I2 = c.i1, Q2 = c.q1;
    c.i1 = I_P; c.q1 = Q_P;
    const double cross = c.i1 * Q2 - I2 * c.q1;
    const double dot = fabs(c.i1 * I2 + c.q1 * Q2);
    const double freq_err = atan2(cross, dot) / M_PI;
    carr_err = atan(Q_P / I_P) / (2.0 * M_PI);
    const double carr_nco = c.old_carr_nco + p.k1 * carr_err - p.k2 * c.old_carr_error -
                            p.k3 * freq_err;
    c.old_carr_nco = carr_nco;
    c.old_carr_error = carr_err;
    c.carr_freq = c.carr_freq_basis + carr_nco;
    // DLL (tracking.sci:355-374)
    const double aEm = sqrt(I_E * I_E + Q_E * Q_E), aLm = sqrt(I_L * I_L + Q_L * Q_L);
    code_err = (aEm - aLm) / (aEm + aLm);
    const double code_nco = c.old_code_nco + (p.tau2 / p.tau1) * (code_err - c.old_code_error) +
                            code_err * (p.pdi_code / p.tau1);
    c.old_code_nco = code_nco;
    c.old_code_error = code_err;
    if (p.code_nco_variant == 1) {
      c.code_freq = p.code_basis - code_nco;               // :366, no carrier aiding
    } else if (p.system == 1) {
      const double fch = (double)c.code_id;                // :367-370
      c.code_freq = p.code_basis - code_nco +
                    (c.carr_freq - (p.if_freq + p.l1_if_step * fch)) /
                        ((p.glo_zero + fch * p.l1_if_step) / p.code_basis);
    } else {
      c.code_freq = p.code_basis - code_nco + ((c.carr_freq - p.if_freq) / 1540);
    }
  }
  c.n_epochs++;
  gnsscorr_sgt_epoch r;
  r.i_e = I_E; r.i_p = I_P; r.i_l = I_L; r.q_e = Q_E; r.q_p = Q_P; r.q_l = Q_L;
  r.carr_freq = c.carr_freq;
  r.code_freq = c.code_freq;
  // :379 mtell(fid)/dataAdaptCoeff (the whole-sample position after the read)
  // or :384 currentSample/dataAdaptCoeff - remCodePhase*(fs/1000)/codeLength
  r.absolute_sample = p.abs_sample_variant == 1
                          ? (double)c.pos
                          : (double)c.pos - c.rem_code * (p.fs / 1000) / dL;
  r.dll_discr = code_err;
  r.dll_discr_filt = c.old_code_nco;
  r.pll_discr = carr_err;
  r.pll_discr_filt = c.old_carr_nco;
  r.blksize = (int32_t)blk;
  r.status = 0;
  return r;
}

__device__ __forceinline__ int xcd_channel(int b, int G) {
  const int q = G >> 3, r = G & 7, x = b & 7, slot = b >> 3;
  return x * q + (x < r ? x : r) + slot;
}

// indices are in [0, L+1] for every state the loop produces (remCode in
// [0, step)); the clamp only keeps a corrupted state inside the LDS table, in
// one instruction: a negative index wraps to a huge unsigned and lands on hi
__device__ __forceinline__ int clampu(int i, int hi) { return (int)min((unsigned)i, (unsigned)hi); }

// a value every lane of the workgroup holds (the channel's state is uniform):
// held in scalar registers instead of a VGPR pair
__device__ __forceinline__ double uni(double v) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((int)b);
  const unsigned hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// wave total, uniform: DPP row_shr 1/2/4/8 (a Hillis-Steele scan in each
// 16-lane row, 0.0 shifted in) leaves each row's sum in its lane 15 and the
// four rows add in scalar registers -- VALU only, where a 64-bit __shfl_xor
// butterfly is two ds_bpermute round trips per step.  Every lane must be active.
template <int CTRL>
__device__ __forceinline__ double dpp_shr(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_f64(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_shr<0x111>(v);
  v += dpp_shr<0x112>(v);
  v += dpp_shr<0x114>(v);
  v += dpp_shr<0x118>(v);
  return (lane_f64(v, 15) + lane_f64(v, 31)) + (lane_f64(v, 47) + lane_f64(v, 63));
}

// WAVE: one wavefront per channel (many-channel launches): the butterfly sums
// leave the totals in every lane, so an epoch needs no LDS partials and no
// barrier, and the loop filters run once per wave instead of once per wave of
// a 4-16-wave workgroup.
// MAXT: the launch bound (64 = WAVE; 256 for the default small-receiver shape,
// which then keeps its registers instead of fitting the 1024-thread budget).
// Wave mode asks for 3 waves per SIMD (<= 168 VGPRs): measured 3 % faster than
// the 2 the chunked path otherwise compiles to.
template <int FT, bool CLOSED, int MAXT>
// (with the prefix columns a wave-mode workgroup takes 16 KiB + the code table:
// 7 fit a CU for GLONASS (511 chips, 4112 B table), 6 for GPS (1023 chips, 8208 B);
// that is under 2 waves per SIMD, so the bound asks for 2)
__global__ __launch_bounds__(MAXT, MAXT == 64 ? (sgt_prefix(64) ? 2 : SGT_WPE) : 1) void sgt_track_kernel(
    SgtParams p, const int8_t* __restrict__ ifbuf, int64_t stride, int64_t n_samples,
    const uint32_t* __restrict__ codes, gnsscorr_sgt_chan* __restrict__ chans, int n_epochs,
    gnsscorr_sgt_epoch* __restrict__ out) {
#pragma clang fp contract(off)
  // the code as +-1.0 (E/P/L accumulate with one fma), L + 2 entries: dynamic,
  // so a 511-chip GLONASS table takes 4.1 KB, not the 1023-chip maximum
  extern __shared__ double s_sgn[];
  __shared__ double s_part[2][kMaxWaves][6];
  __shared__ double2 s_w[40];   // chunked paths: exp(i*A*n/fs), n < kC
  const int ch = xcd_channel(blockIdx.x, gridDim.x);
  constexpr bool WAVE = MAXT == 64;
  constexpr bool kPrefix = sgt_prefix(MAXT);
  const int T = WAVE ? 64 : blockDim.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // this lane's prefix column (kPrefix): entry m at s_pf[m * 64]
  double2* s_pf = reinterpret_cast<double2*>(reinterpret_cast<uint8_t*>(s_sgn) +
                                             sgt_tab_bytes(p.code_length) +
                                             (size_t)wave * kPfWaveBytes) + lane;
  const int nw = T >> 6;
  gnsscorr_sgt_chan c = chans[ch];
  const int L = p.code_length;
  const int row = p.system == 1 ? 0 : c.code_id;
  for (int i = tid; i < L + 2; i += T) {
    s_sgn[i] = codes[row * kPadLen + i] ? -1.0 : 1.0;   // sign-bit masks of the table
  }
  // one guard entry past the padded table (a copy of entry L+1): the unclamped
  // in_table path relies on a rounding argument to stay within [0, L+1]
  if (tid == 0) s_sgn[L + 2] = codes[row * kPadLen + L + 1] ? -1.0 : 1.0;
  __syncthreads();

  const int8_t* base = ifbuf + (int64_t)c.stream * stride;
  const double dL = (double)L;
  int e = 0;
  for (; e < n_epochs; e++) {
    gnsscorr_sgt_epoch* rec = out + (int64_t)ch * n_epochs + e;
    if (c.status != 0) {
      if (tid == 0) { gnsscorr_sgt_epoch z = {}; z.status = 1; *rec = z; }
      continue;
    }
    const double step = c.code_freq / p.fs;
    const double blk_d = ceil((dL - c.rem_code) / step);
    // tracking.sci:273-277: not enough samples (NaN or huge blksize from a
    // corrupted state stops too, as does a blksize of 2^31 or more)
    if (!(blk_d <= (double)(n_samples - c.pos) && blk_d < 2147483648.0)) {
      c.status = 1;
      if (tid == 0) {
        gnsscorr_sgt_epoch z = {};
        z.status = 1;
        z.blksize = blk_d >= 0.0 && blk_d < 2147483648.0 ? (int32_t)blk_d : -1;
        *rec = z;
      }
      continue;
    }
    const int blk = (int)blk_d;
    const double aE = c.rem_code - p.spc, aL = c.rem_code + p.spc, aP = c.rem_code;
    const double A = (c.carr_freq * 2.0) * M_PI;        // (carrFreq * 2.0 * %pi)
    double ie = 0, ip = 0, il = 0, qe = 0, qp = 0, ql = 0;
    const int8_t* src = base + (FT == 2 ? 2 : 1) * c.pos;
    // I/Q byte order as bit-field offsets (switchIQ without a per-sample select)
    const int sh_re = p.switch_iq ? 8 : 0, sh_im = 8 - sh_re;
    // kU samples per thread per pass.  The IF words of pass n+1 are loaded
    // while pass n is processed (with a plain unrolled loop the compiler kept
    // one load in flight and waited on memory latency at every sample); the
    // last, partial pass is guarded per sample.
    constexpr int kU = 8;
    auto load = [&](int k) -> int {
      if (FT == 2) return *reinterpret_cast<const uint16_t*>(src + 2 * k);
      return src[k];
    };
    // Every code index lies in [0, L+1] (the padded table) when remCode >= spc - 1
    // (aE > -1) and spc < 0.99: blksize = ceil((L - remCode)/step) keeps
    // (blksize-1)*step below L - remCode up to rounding, so aL + t < L + 1.  The
    // loop keeps remCode in [0, step); only a state set from outside can fail
    // the test, and then the indices are clamped into the table (kClamp).
    const bool in_table = c.rem_code >= p.spc - 1.0 && p.spc >= 0.0 && p.spc < 0.99;
    auto run = [&](auto clamp_tag) {
    constexpr bool kClamp = decltype(clamp_tag)::value;
    // carrier at the thread's first sample, rotation by T samples
    const double th0 = A * ((double)tid / p.fs) + c.rem_carr, thw = A * ((double)T / p.fs);
    double sn, cs, sw, cw;
    sincos(th0, &sn, &cs);   // one shared argument reduction per angle
    sincos(thw, &sw, &cw);   // (sgt.o is built with promote-alloca-to-lds off)
    auto index = [&](double x) {
      const int i = (int)ceil(x);
      return kClamp ? clampu(i, L + 1) : i;
    };
    auto sample = [&](int k, int w) {
      const double t = (double)k * step;
      const double gE = s_sgn[index(aE + t)];
      const double gP = s_sgn[index(aP + t)];
      const double gL = s_sgn[index(aL + t)];
      double re, im;
      if (FT == 2) {
        re = (double)(int)__builtin_amdgcn_sbfe(w, sh_re, 8);   // (the builtin is typed unsigned)
        im = (double)(int)__builtin_amdgcn_sbfe(w, sh_im, 8);
      } else {
        re = (double)w;
        im = 0.0;
      }
      // (explicit fma: the carrier and the sums only need fp64 accuracy; the
      // code indices above stay uncontracted and bit-exact)
      const double qb = fma(cs, re, -(sn * im));   // real(carrsig .* rawSignal)
      const double ib = fma(cs, im, sn * re);      // imag(carrsig .* rawSignal)
      ie = fma(ib, gE, ie); ip = fma(ib, gP, ip); il = fma(ib, gL, il);   // +-ib exactly
      qe = fma(qb, gE, qe); qp = fma(qb, gP, qp); ql = fma(qb, gL, ql);
      const double c2 = fma(cs, cw, -(sn * sw));
      sn = fma(sn, cw, cs * sw);
      cs = c2;
    };
    const int n_full = blk / (kU * T);   // passes whose kU samples all exist for every thread
    int k0 = tid;
    int w[kU];
    if (n_full > 0) {
#pragma unroll
      for (int u = 0; u < kU; u++) w[u] = load(k0 + u * T);
    }
    for (int n = 0; n < n_full; n++, k0 += kU * T) {
      int cur[kU];
#pragma unroll
      for (int u = 0; u < kU; u++) cur[u] = w[u];
      if (n + 1 < n_full) {
#pragma unroll
        for (int u = 0; u < kU; u++) w[u] = load(k0 + kU * T + u * T);
      }
#pragma unroll
      for (int u = 0; u < kU; u++) sample(k0 + u * T, cur[u]);
    }
    // the remainder: fewer than kU * T samples
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int k = k0 + u * T;
      w[u] = k < blk ? load(k) : 0;
    }
#pragma unroll
    for (int u = 0; u < kU; u++) {
      const int k = k0 + u * T;
      if (k < blk) sample(k, w[u]);
    }
    };
    // ---- chunked path (round 3).  A lane takes chunks of kC consecutive
    // samples (chunk q at k = q*kC - mis, q = lane + j*T, one or two 16-byte
    // loads on the 16-byte grid of the stream) instead of single samples
    // strided by T.  Within a chunk each code index takes at most two values
    // ((kC-1)*step < 1): the index j0 of the chunk's first sample comes from
    // the exact formula, and the first sample of index j0+1 from the crossing
    // d = (j0 - a)/step (sample k has index > j0 iff a + k*step > j0, i.e.
    // k > d).  When d lies within 1e-6 samples of an integer the real-valued
    // crossing could round either way, so that lane recomputes the chunk's
    // crossings with the exact fp64 indices, sample by sample.  Samples then
    // select the code by position (n < beta ? c(j0) : c(j0+1)) instead of
    // evaluating ceil(rem -/+ spc + k*step) three times each.
    // Carrier: exp(i theta_k) = exp(i theta_k0) * W_n, n = k - k0; W_n =
    // exp(i*A*n/fs) (n < kC) is an LDS table read by broadcast, each arm sums
    // code * W_n * raw over the chunk and rotates the sum by exp(i theta_k0)
    // once per chunk (tracking.sci:305-326, same sums up to fp64 rounding).
    constexpr int kBps = FT == 2 ? 2 : 1;
    auto run_chunks = [&](auto kc_tag) {
      constexpr int kC = decltype(kc_tag)::value;
      const int mis = (int)((uintptr_t)src & 15) / kBps;
      const uint4* ab = reinterpret_cast<const uint4*>(src - mis * kBps);
      const int nC = (blk + mis + kC - 1) / kC;
      const int nIt = (nC + T - 1) / T;
      const double inv_step = uni(1.0 / step), stp = uni(step);
      const double aX[3] = {uni(aE), uni(aP), uni(aL)};
      double sb, cb, sR, cR;
      sincos(A * ((double)(tid * kC - mis) / p.fs) + c.rem_carr, &sb, &cb);
      double swl = 0.0, cwl = 1.0;
      if (WAVE || tid < kC) sincos(A * ((double)tid / p.fs), &swl, &cwl);   // W_tid
      if (tid < kC) s_w[tid] = make_double2(cwl, swl);
      if constexpr (WAVE) {
        // the rotation by T*kC samples without a third sincos: lanes 63 and 0
        // hold the carrier at k = 63 kC - mis and -mis, lane kC holds W_kC, so
        // exp(i A 64 kC / fs) = e(63) * conj(e(0)) * W_kC (fp64 rounding only)
        const double c63 = lane_f64(cb, 63), s63 = lane_f64(sb, 63);
        const double c0 = lane_f64(cb, 0), s0 = lane_f64(sb, 0);
        const double cK = lane_f64(cwl, kC), sK = lane_f64(swl, kC);
        const double dc = fma(c63, c0, s63 * s0), ds = fma(s63, c0, -(c63 * s0));
        cR = fma(dc, cK, -(ds * sK));
        sR = fma(dc, sK, ds * cK);
      } else {
        sincos(A * ((double)(T * kC) / p.fs), &sR, &cR);
        sR = uni(sR);
        cR = uni(cR);
      }
      __syncthreads();
      double accI[3] = {0.0, 0.0, 0.0}, accQ[3] = {0.0, 0.0, 0.0};
      constexpr int kW = kC * kBps / 16;   // 16-byte words per chunk
      uint4 nx[kW];
      auto fetch = [&](int it, uint4 (&x)[kW]) {
        const int q = it * T + tid;
#pragma unroll
        for (int u = 0; u < kW; u++) {
          // only words holding a sample of the epoch: none past the stream's end
          const int ks = q * kC - mis + u * (16 / kBps);
          x[u] = ks < blk ? ab[q * kW + u] : make_uint4(0, 0, 0, 0);
        }
      };
      fetch(0, nx);
      for (int it = 0; it < nIt; it++) {
        uint32_t wd[4 * kW];
#pragma unroll
        for (int u = 0; u < kW; u++) {
          wd[4 * u] = nx[u].x; wd[4 * u + 1] = nx[u].y;
          wd[4 * u + 2] = nx[u].z; wd[4 * u + 3] = nx[u].w;
        }
        if (it + 1 < nIt) fetch(it + 1, nx);
        const int q = it * T + tid;
        const int k0 = q * kC - mis;
        // the epoch's first and last chunks: samples outside [0, blk) count as 0
        if (k0 < 0 || k0 + kC > blk) {
#pragma unroll
          for (int n = 0; n < kC; n++) {
            const bool v = (unsigned)(k0 + n) < (unsigned)blk;
            constexpr int kSpw = 4 / kBps;   // samples per dword
            const uint32_t m = (kBps == 2 ? 0xffffu : 0xffu) << (8 * kBps * (n % kSpw));
            wd[n / kSpw] &= v ? 0xffffffffu : ~m;
          }
        }
        const double t0 = (double)k0 * stp;
        int beta[3], j0[3];
        double g0[3], g1[3];
        bool risky = false;
#pragma unroll
        for (int x = 0; x < 3; x++) {
          const double jf = ceil(aX[x] + t0);
          j0[x] = (int)jf;
          const double d = (jf - aX[x]) * inv_step;
          const double fd = floor(d);
          const double fr = d - fd;
          risky |= !(fr > 1e-6 && fr < 1.0 - 1e-6);
          beta[x] = min(max((int)fd + 1 - k0, 1), kC);
          // the code as +-1.0: only the high word differs (the low one is 0)
          const uint32_t* sg = reinterpret_cast<const uint32_t*>(s_sgn) + 1;
          g0[x] = __longlong_as_double((long long)sg[2 * clampu(j0[x], L + 1)] << 32);
          g1[x] = __longlong_as_double((long long)sg[2 * clampu(j0[x] + 1, L + 1)] << 32);
        }
        if (risky && q < nC) {
          // exact crossings: the first sample whose index exceeds j0
#pragma unroll 1
          for (int x = 0; x < 3; x++) {
            int b = kC;
#pragma unroll 1
            for (int n = kC - 1; n >= 1; n--)
              if ((int)ceil(aX[x] + (double)(k0 + n) * stp) > j0[x]) b = n;
            beta[x] = b;
          }
        }
        double Ur[3] = {0.0, 0.0, 0.0}, Ui[3] = {0.0, 0.0, 0.0};
        // the W_n reads are loop invariant: an opaque offset per chunk keeps
        // them from being hoisted out of the chunk loop (16 complex in VGPRs)
        int wo = 0;
        asm volatile("" : "+v"(wo));
        if constexpr (kPrefix) {
          // U_x = g1 T + (g0 - g1) B_x per sub-block: T its sum of W_n*raw, B_x
          // the sum over its samples before arm x's crossing (a prefix read
          // back from LDS at the crossing); g0 - g1 is 0 or +-2, exact
          double dg[3];
#pragma unroll
          for (int x = 0; x < 3; x++) dg[x] = g0[x] - g1[x];
#pragma unroll
          for (int h = 0; h < kC / kSub; h++) {
            double Pr = 0.0, Pi = 0.0;
#pragma unroll
            for (int m = 0; m < kSub; m++) {
              const int n = h * kSub + m;
              double ur, ui;
              if constexpr (FT == 2) {
                const uint32_t w = wd[n >> 1];
                const int sh = (n & 1) * 16;
                const double re = (double)(int)__builtin_amdgcn_sbfe(w, sh + sh_re, 8);
                const double im = (double)(int)__builtin_amdgcn_sbfe(w, sh + sh_im, 8);
                const double2 W = s_w[n + wo];   // broadcast read
                ur = fma(W.x, re, -(W.y * im));
                ui = fma(W.x, im, W.y * re);
              } else {
                const double re = (double)(int)__builtin_amdgcn_sbfe(wd[n >> 2], (n & 3) * 8, 8);
                const double2 W = s_w[n + wo];
                ur = W.x * re;
                ui = W.y * re;
              }
              Pr += ur;
              Pi += ui;
              s_pf[m * 64] = make_double2(Pr, Pi);
            }
#pragma unroll
            for (int x = 0; x < 3; x++) {
              const int bl = beta[x] - h * kSub;   // this sub-block's samples before the crossing
              const double2 B = s_pf[min(max(bl - 1, 0), kSub - 1) * 64];
              const double br = bl > 0 ? B.x : 0.0, bi = bl > 0 ? B.y : 0.0;
              Ur[x] = fma(dg[x], br, fma(g1[x], Pr, Ur[x]));
              Ui[x] = fma(dg[x], bi, fma(g1[x], Pi, Ui[x]));
            }
          }
        } else
#pragma unroll
        for (int n = 0; n < kC; n++) {
          double ur, ui;
          if constexpr (FT == 2) {
            const uint32_t w = wd[n >> 1];
            const int sh = (n & 1) * 16;
            const double re = (double)(int)__builtin_amdgcn_sbfe(w, sh + sh_re, 8);
            const double im = (double)(int)__builtin_amdgcn_sbfe(w, sh + sh_im, 8);
            const double2 W = s_w[n + wo];   // broadcast read
            ur = fma(W.x, re, -(W.y * im));   // W_n * raw
            ui = fma(W.x, im, W.y * re);
          } else {
            const double re = (double)(int)__builtin_amdgcn_sbfe(wd[n >> 2], (n & 3) * 8, 8);
            const double2 W = s_w[n + wo];
            ur = W.x * re;
            ui = W.y * re;
          }
#pragma unroll
          for (int x = 0; x < 3; x++) {
            const double g = n < beta[x] ? g0[x] : g1[x];
            Ur[x] = fma(ur, g, Ur[x]);
            Ui[x] = fma(ui, g, Ui[x]);
          }
#ifdef SGT_SCHED
          if (n % SGT_SCHED == SGT_SCHED - 1) __builtin_amdgcn_sched_barrier(0);
#endif
        }
        // exp(i theta_k0) * U: real part -> Q (qBasebandSignal), imaginary -> I
#pragma unroll
        for (int x = 0; x < 3; x++) {
          accQ[x] = fma(cb, Ur[x], fma(-sb, Ui[x], accQ[x]));
          accI[x] = fma(sb, Ur[x], fma(cb, Ui[x], accI[x]));
        }
        const double cn = fma(cb, cR, -(sb * sR));
        sb = fma(sb, cR, cb * sR);
        cb = cn;
      }
      ie = accI[0]; ip = accI[1]; il = accI[2];
      qe = accQ[0]; qp = accQ[1]; ql = accQ[2];
    };
    // ---- chip-aligned chunks (round 5; every launch shape).  Thread chunk q holds
    // the samples of ONE prompt chip j = jF + q, k in [kS(j), kS(j+1)), kS(j) the
    // first sample whose prompt index ceil(remCode + k*step) reaches j.  Within
    // it the prompt code is constant, the early arm (remCode - spc) is still on
    // chip j-1 for its first bE samples and the late arm (remCode + spc) already
    // on chip j+1 from sample bL on; bE, bL take one of two values each (floor
    // of spc/step or one more), so with T the chunk's sum of W_n * raw,
    // H = T after bE samples and G = T after bL samples (captured in two short
    // windows of the sample loop):
    //   U_P = c(j) T,  U_E = c(j) T + (c(j-1) - c(j)) H,
    //   U_L = c(j) T + (c(j+1) - c(j)) (T - G)                 (tracking.sci:316-326)
    // No per-sample code selects and no prefix columns in LDS (the wave kernel's
    // LDS is the code table and the W_n table).  The chunk's IF bytes start
    // anywhere: kNW dwords are loaded and realigned by v_alignbyte.  The carrier
    // at a chunk's first sample comes from the thread's previous chunk (T chips
    // earlier: kS moves by m or m + 1 samples) times a uniform rotation.
    // Lanes whose chunk falls outside the windows (exact crossings moved by
    // rounding) take an exact per-sample loop for that chunk.
    auto run_chips = [&](auto kc_tag) {
      constexpr int kC = decltype(kc_tag)::value;   // 16, 17, 32 or 33: longest chunk
      constexpr int kHW = 5, kTW = 9;               // capture windows: n < kHW, n >= kC - kTW
      constexpr int kNR = (kC * kBps + 3) / 4;      // realigned dwords holding kC samples
      constexpr int kNW = kNR + 1;                  // loaded dwords (any byte alignment)
      const double inv_step = uni(1.0 / step), stp = uni(step);
      const double aPu = uni(aP), aEu = uni(aE), aLu = uni(aL);
      const int jF = (int)ceil(aPu);                                     // k = 0's prompt chip
      const int nC = (int)ceil(aPu + (double)(blk - 1) * stp) - jF + 1;  // chips of the epoch
      const int nIt = (nC + T - 1) / T;
      const int m64 = (int)floor((double)T * inv_step);                  // samples per T chips
      {
        double sw, cw;
        sincos(A * ((double)tid / p.fs), &sw, &cw);
        if (tid < kC) s_w[tid] = make_double2(cw, sw);
      }
      double sR, cR;   // exp(i A m64 / fs): the carrier T chips on
      sincos(A * ((double)m64 / p.fs), &sR, &cR);
      sR = uni(sR);
      cR = uni(cR);
      __syncthreads();
      // first k with ceil(a + k*step) >= t: exact when the real-valued estimate
      // has a 1e-6-sample margin from an integer; else one of est - 1, est, est + 1
      auto first_k = [&](double a, int t, bool& risky) -> int {
        const double d = ((double)(t - 1) - a) * inv_step;
        const double fd = floor(d);
        const double fr = d - fd;
        risky |= !(fr > 1e-6 && fr < 1.0 - 1e-6);
        return (int)fd + 1;
      };
      auto exact_k = [&](double a, int t, int est) -> int {
        if ((int)ceil(a + (double)(est - 1) * stp) >= t) return est - 1;
        if ((int)ceil(a + (double)est * stp) >= t) return est;
        return est + 1;
      };
      struct Bd { int kS, kN, kE, kL; };
      auto bounds = [&](int j) {
        bool risky = false;
        Bd b;
        b.kS = first_k(aPu, j, risky);
        b.kN = first_k(aPu, j + 1, risky);
        b.kE = first_k(aEu, j, risky);
        b.kL = first_k(aLu, j + 1, risky);
        if (risky) {
          b.kS = exact_k(aPu, j, b.kS);
          b.kN = exact_k(aPu, j + 1, b.kN);
          b.kE = exact_k(aEu, j, b.kE);
          b.kL = exact_k(aLu, j + 1, b.kL);
        }
        return b;
      };
      typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
      auto fetch = [&](const Bd& b, uint32_t (&w)[kNW]) {
        const uintptr_t a0 = (uintptr_t)(src + (int64_t)kBps * b.kS);
        const uint32_t* p4 = reinterpret_cast<const uint32_t*>(a0 & ~(uintptr_t)3);
        // a wave whose lanes all read inside the epoch loads without guards
        const bool inside = b.kS >= 0 && b.kS + (4 * kNW + kBps - 1) / kBps <= blk;
        if (__builtin_amdgcn_ballot_w64(!inside) == 0) {
#pragma unroll
          for (int u = 0; u + 4 <= kNW; u += 4) {
            const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(p4 + u);
            w[u] = v.x; w[u + 1] = v.y; w[u + 2] = v.z; w[u + 3] = v.w;
          }
#pragma unroll
          for (int u = kNW & ~3; u < kNW; u++) w[u] = p4[u];
        } else {
          // only dwords holding a byte of the epoch [src, src + kBps blk)
          const uintptr_t lo = (uintptr_t)src, hi = lo + (uintptr_t)((int64_t)kBps * blk);
#pragma unroll
          for (int u = 0; u < kNW; u++) {
            const uintptr_t a = (uintptr_t)(p4 + u);
            w[u] = (a + 4 > lo && a < hi) ? p4[u] : 0u;
          }
        }
      };
      double accI[3] = {0.0, 0.0, 0.0}, accQ[3] = {0.0, 0.0, 0.0};
      const uint32_t* sg = reinterpret_cast<const uint32_t*>(s_sgn) + 1;   // hi words
      auto code = [&](int i) {   // the code as +-1.0 (only the high word differs)
        return __longlong_as_double((long long)sg[2 * clampu(i, L + 1)] << 32);
      };
      Bd b = bounds(jF + tid);
      double sb, cb;   // carrier at the chunk's first sample
      sincos(A * ((double)b.kS / p.fs) + c.rem_carr, &sb, &cb);
      uint32_t nx[kNW];
      if (SGT_CHIP_PF) fetch(b, nx);
      for (int it = 0; it < nIt; it++) {
        uint32_t w[kNW];
        if (!SGT_CHIP_PF) fetch(b, nx);
#pragma unroll
        for (int u = 0; u < kNW; u++) w[u] = nx[u];
        const int j = jF + it * T + tid;
        Bd bn = b;
        if (it + 1 < nIt) {
          bn = bounds(j + T);
          if (SGT_CHIP_PF) fetch(bn, nx);
        }
        const int len = b.kN - b.kS, bE = b.kE - b.kS, bL = b.kL - b.kS;
        const bool ok = len <= kC && len >= kC - 3 && bE >= 0 && bE <= kHW && bL - 1 >= kC - kTW &&
                        bL <= len;
        // the chunk's samples from byte a0 & 3 on, realigned to dword 0
        const uint32_t sh = (uint32_t)((uintptr_t)(src + (int64_t)kBps * b.kS) & 3);
        uint32_t r[kNR];
#pragma unroll
        for (int u = 0; u < kNR; u++) r[u] = __builtin_amdgcn_alignbyte(w[u + 1], w[u], sh);
        // samples outside [0, blk) count as 0 (the epoch's first and last chunks)
        const bool edge = b.kS < 0 || b.kS + kC > blk;
        const bool any_edge = __builtin_amdgcn_ballot_w64(edge) != 0;
        double Tr = 0.0, Ti = 0.0, Hr = 0.0, Hi = 0.0, Gr = 0.0, Gi = 0.0;
        auto sample_loop = [&](auto edge_tag) {
          constexpr bool kEdge = decltype(edge_tag)::value;
          int wo = 0;   // opaque: the W_n reads stay inside the loop
          asm volatile("" : "+v"(wo));
#pragma unroll
          for (int n = 0; n < kC; n++) {
            if (n % SGT_CHIP_GROUP == 0 && n > 0) {
              // groups of samples: the next group's W_n reads and IF words depend
              // on the running sum so far, so the compiler cannot hoist every
              // sample's table entry and conversion to the chunk's start
              asm volatile("" : "+v"(wo) : "v"(Tr));
#pragma unroll
              for (int u = n * kBps / 4; u < kNR && u < (n + SGT_CHIP_GROUP) * kBps / 4 + 1; u++)
                asm volatile("" : "+v"(r[u]) : "v"(Ti));
            }
            int re, im = 0;
            if constexpr (FT == 2) {
              re = (int)__builtin_amdgcn_sbfe(r[n >> 1], (n & 1) * 16 + sh_re, 8);
              im = (int)__builtin_amdgcn_sbfe(r[n >> 1], (n & 1) * 16 + sh_im, 8);
            } else {
              re = (int)__builtin_amdgcn_sbfe(r[n >> 2], (n & 3) * 8, 8);
            }
            bool v = true;
            if (n >= kC - 3) v = n < len;
            if (kEdge) v = v && (unsigned)(b.kS + n) < (unsigned)blk;
            if (kEdge || n >= kC - 3) {
              re = v ? re : 0;
              im = v ? im : 0;
            }
            const double2 W = s_w[n + wo];   // broadcast read
            if constexpr (SGT_CHIP_FMA) {
              // T += W_n * raw as fused steps (fp64 rounding only)
              Tr = fma(W.x, (double)re, Tr);
              Ti = fma(W.y, (double)re, Ti);
              if constexpr (FT == 2) {
                Tr = fma(-W.y, (double)im, Tr);
                Ti = fma(W.x, (double)im, Ti);
              }
            } else {
              double ur, ui;
              if constexpr (FT == 2) {
                ur = fma(W.x, (double)re, -(W.y * (double)im));   // W_n * raw
                ui = fma(W.x, (double)im, W.y * (double)re);
              } else {
                ur = W.x * (double)re;
                ui = W.y * (double)re;
              }
              Tr += ur;
              Ti += ui;
            }
            if (n < kHW) {
              const bool h = n == bE - 1;
              Hr = h ? Tr : Hr;
              Hi = h ? Ti : Hi;
            }
            if (n >= kC - kTW) {
              const bool g = n == bL - 1;
              Gr = g ? Tr : Gr;
              Gi = g ? Ti : Gi;
            }
          }
        };
        if (any_edge) sample_loop(std::true_type{});
        else sample_loop(std::false_type{});
        if (ok) {
          const double cP = code(j), dE = code(j - 1) - cP, dL = code(j + 1) - cP;   // dE, dL: 0, +-2
          const double PTr = cP * Tr, PTi = cP * Ti;
          const double Ur[3] = {fma(dE, Hr, PTr), PTr, fma(dL, Tr - Gr, PTr)};
          const double Ui[3] = {fma(dE, Hi, PTi), PTi, fma(dL, Ti - Gi, PTi)};
#pragma unroll
          for (int x = 0; x < 3; x++) {
            accQ[x] = fma(cb, Ur[x], fma(-sb, Ui[x], accQ[x]));
            accI[x] = fma(sb, Ur[x], fma(cb, Ui[x], accI[x]));
          }
        } else {
          // exact per-sample loop for this lane's chunk (rare)
#pragma unroll 1
          for (int k = max(b.kS, 0); k < min(b.kN, blk); k++) {
            const double t = (double)k * stp;
            const double gx[3] = {s_sgn[clampu((int)ceil(aEu + t), L + 1)],
                                  s_sgn[clampu((int)ceil(aPu + t), L + 1)],
                                  s_sgn[clampu((int)ceil(aLu + t), L + 1)]};
            double re, im = 0.0;
            if constexpr (FT == 2) {
              const int wv = *reinterpret_cast<const uint16_t*>(src + 2 * (int64_t)k);
              re = (double)(int)__builtin_amdgcn_sbfe(wv, sh_re, 8);
              im = (double)(int)__builtin_amdgcn_sbfe(wv, sh_im, 8);
            } else {
              re = (double)src[k];
            }
            double se, ce;
            sincos(A * ((double)k / p.fs) + c.rem_carr, &se, &ce);
            const double qb = fma(ce, re, -(se * im)), ib = fma(ce, im, se * re);
#pragma unroll
            for (int x = 0; x < 3; x++) {
              accQ[x] = fma(qb, gx[x], accQ[x]);
              accI[x] = fma(ib, gx[x], accI[x]);
            }
          }
        }
        if (it + 1 < nIt) {
          // carrier at the next chunk (T chips on): kS moves by m64 or m64 + 1 samples
          const int D = bn.kS - b.kS;
          if (D == m64 || D == m64 + 1) {
            double rc = cR, rs = sR;
            if (D != m64) {
              const double2 W1 = s_w[1];
              rc = fma(cR, W1.x, -(sR * W1.y));
              rs = fma(sR, W1.x, cR * W1.y);
            }
            const double cn = fma(cb, rc, -(sb * rs));
            sb = fma(sb, rc, cb * rs);
            cb = cn;
          } else {
            sincos(A * ((double)bn.kS / p.fs) + c.rem_carr, &sb, &cb);
          }
          b = bn;
        }
      }
      ie = accI[0]; ip = accI[1]; il = accI[2];
      qe = accQ[0]; qp = accQ[1]; ql = accQ[2];
    };
    const bool chunked = p.chunked && in_table && 15.0 * step < 0.999 &&
                         ((uintptr_t)src & (kBps - 1)) == 0;
    const double invs = 1.0 / step, sps = floor(p.spc * invs);   // samples per chip, spc in samples
    // the longest chunk is floor(samples per chip) + 1 samples: kC = 16 / 17 (GPS
    // at 16 / 16.368 Msps), 32 / 33 (GLONASS); the loop masks its last 3 samples
    const int ipc = (SGT_CHIPS && MAXT <= 256 && chunked && sps <= 3.0 && invs < 33.0) ? (int)invs : 0;
    const int kcs = ipc >= 29 ? (ipc >= 32 ? 33 : 32) : (ipc >= 13 && ipc <= 16 ? (ipc >= 16 ? 17 : 16) : 0);
    if (kcs) {
      if (kcs == 33) run_chips(std::integral_constant<int, 33>{});
      else if (kcs == 32) run_chips(std::integral_constant<int, 32>{});
      else if (kcs == 17) run_chips(std::integral_constant<int, 17>{});
      else run_chips(std::integral_constant<int, 16>{});
    }
    else if (chunked && SGT_KC32 && 31.0 * step < 0.999)
      run_chunks(std::integral_constant<int, 32>{});
    else if (chunked)
      run_chunks(std::integral_constant<int, 16>{});
    else if (in_table)
      run(std::false_type{});
    else
      run(std::true_type{});
    ie = wave_sum(ie); ip = wave_sum(ip); il = wave_sum(il);
    qe = wave_sum(qe); qp = wave_sum(qp); ql = wave_sum(ql);
    double S[6] = {ie, ip, il, qe, qp, ql};
    if constexpr (!WAVE) {
      const int par = e & 1;
      if (lane == 0) {
        s_part[par][wave][0] = ie; s_part[par][wave][1] = ip; s_part[par][wave][2] = il;
        s_part[par][wave][3] = qe; s_part[par][wave][4] = qp; s_part[par][wave][5] = ql;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 6; j++) S[j] = 0.0;
      for (int w = 0; w < nw; w++)
#pragma unroll
        for (int j = 0; j < 6; j++) S[j] += s_part[par][w][j];
    }
    const gnsscorr_sgt_epoch r = sgt_epoch_end<CLOSED>(p, c, blk, step, S);
    if (tid == 0) *rec = r;
  }
  if (tid == 0) chans[ch] = c;
}

// The loop half alone: each thread runs one channel's epochs on given sums
// (sums[(ch*n_epochs + e)*6 + j]) instead of correlations of a record.  No
// record bounds (there is no record); a NaN / negative / >= 2^31 blksize stops
// the channel as in the tracking kernel.
__global__ void sgt_replay_kernel(SgtParams p, gnsscorr_sgt_chan* __restrict__ chans, int n_ch,
                                  int n_epochs, const double* __restrict__ sums,
                                  gnsscorr_sgt_epoch* __restrict__ out) {
#pragma clang fp contract(off)
  const int ch = blockIdx.x * blockDim.x + threadIdx.x;
  if (ch >= n_ch) return;
  gnsscorr_sgt_chan c = chans[ch];
  for (int e = 0; e < n_epochs; e++) {
    gnsscorr_sgt_epoch* rec = out + (int64_t)ch * n_epochs + e;
    if (c.status != 0) {
      gnsscorr_sgt_epoch z = {};
      z.status = 1;
      *rec = z;
      continue;
    }
    const double step = c.code_freq / p.fs;
    const double blk_d = ceil(((double)p.code_length - c.rem_code) / step);
    if (!(blk_d >= 0.0 && blk_d < 2147483648.0)) {
      c.status = 1;
      gnsscorr_sgt_epoch z = {};
      z.status = 1;
      z.blksize = -1;
      *rec = z;
      continue;
    }
    const double* sp = sums + ((int64_t)ch * n_epochs + e) * 6;
    const double S[6] = {sp[0], sp[1], sp[2], sp[3], sp[4], sp[5]};
    *rec = sgt_epoch_end<true>(p, c, (int)blk_d, step, S);
  }
  chans[ch] = c;
}

}  // namespace

// ============================================================================
// host side
// ============================================================================
struct gnsscorr_sgt_ctx {
  gnsscorr_sgt_cfg cfg;
  SgtParams p;
  hipStream_t stream = nullptr;
  uint32_t* d_codes = nullptr;
  gnsscorr_sgt_chan* d_chan = nullptr;
  gnsscorr_sgt_epoch* d_ep = nullptr;
  size_t chan_cap = 0, ep_cap = 0;
};

extern "C" void gnsscorr_sgt_loop_coefs(const gnsscorr_sgt_cfg* cfg, double* tau1, double* tau2,
                                        double* k1, double* k2, double* k3) {
  // calcLoopCoef.sci:39-43 (k = 1.0)
  const double z = cfg->dll_damping;
  const double wn = cfg->dll_noise_bw * 8 * z / (4 * (z * z) + 1);
  *tau1 = 1.0 / (wn * wn);
  *tau2 = 2.0 * z / wn;
  // calcFLLPLLLoopCoef.sci:36-38 (T = PDIcarr = 0.001)
  const double T = 0.001, b = cfg->pll_noise_bw / 0.53;
  *k1 = T * (b * b) + 1.414 * b;
  *k2 = 1.414 * b;
  *k3 = T * (cfg->fll_noise_bw / 0.25);
}

static int check_cfg(const gnsscorr_sgt_cfg* cfg) {
  if (!cfg || (cfg->system != 0 && cfg->system != 1) ||
      (cfg->file_type != 1 && cfg->file_type != 2) || cfg->samp_rate <= 0 ||
      cfg->code_freq_basis <= 0 || cfg->dll_spacing < 0 || cfg->dll_spacing >= 1 ||
      cfg->code_length != (cfg->system == 1 ? 511 : 1023) ||
      (cfg->code_nco_variant != 0 && cfg->code_nco_variant != 1) ||
      (cfg->abs_sample_variant != 0 && cfg->abs_sample_variant != 1)) {
    gnsscorr_set_error("sgt: bad config (system 0/1, file_type 1/2, code_length 1023/511, "
                       "0<=dll_spacing<1, variants 0/1)");
    return GNSSCORR_EINVAL;
  }
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_init_chan(const gnsscorr_sgt_cfg* cfg, int code_id, int stream,
                                      int64_t skip, int64_t code_phase_1b, double acq_freq,
                                      gnsscorr_sgt_chan* o) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (!o || code_phase_1b < 1 || stream < 0 || skip < 0 ||
      (cfg->system == 0 && (code_id < 1 || code_id > 32)) ||
      (cfg->system == 1 && (code_id < -7 || code_id > 6))) {
    gnsscorr_set_error("gnsscorr_sgt_init_chan: bad channel (PRN 1..32 / FCH -7..6, "
                       "code_phase >= 1)");
    return GNSSCORR_EINVAL;
  }
  memset(o, 0, sizeof *o);
  o->code_id = code_id;
  o->stream = stream;
  o->pos = skip + code_phase_1b - 1;   // mseek, tracking.sci:163-168
  o->code_freq = cfg->code_freq_basis;
  o->carr_freq = o->carr_freq_basis = acq_freq;
  o->i1 = o->q1 = 0.001;               // tracking.sci:201
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_destroy(gnsscorr_sgt_ctx* c) {
  if (!c) return GNSSCORR_OK;
  (void)hipSetDevice(c->cfg.device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_codes);
  (void)hipFree(c->d_chan);
  (void)hipFree(c->d_ep);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_create(gnsscorr_sgt_ctx** out, const gnsscorr_sgt_cfg* cfg) {
  if (!out) return GNSSCORR_EINVAL;
  *out = nullptr;
  int rc = check_cfg(cfg);
  if (rc) return rc;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    gnsscorr_set_error("gnsscorr_sgt_create: no HIP device");
    return GNSSCORR_ENODEV;
  }
  if (cfg->device < 0 || cfg->device >= ndev) {
    gnsscorr_set_error("gnsscorr_sgt_create: device %d out of range", cfg->device);
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(cfg->device));
  auto* c = new gnsscorr_sgt_ctx();
  c->cfg = *cfg;
  SgtParams& p = c->p;
  p.system = cfg->system;
  p.file_type = cfg->file_type;
  p.switch_iq = cfg->system == 1 ? cfg->switch_iq : 0;
  p.code_length = cfg->code_length;
  p.code_nco_variant = cfg->code_nco_variant;
  p.abs_sample_variant = cfg->abs_sample_variant;
  // GNSSCORR_SGT_CHUNK=0: the per-sample index path only (A/B and tests)
  const char* chk = getenv("GNSSCORR_SGT_CHUNK");
  p.chunked = !(chk && chk[0] == '0');
  p.fs = cfg->samp_rate;
  p.code_basis = cfg->code_freq_basis;
  p.if_freq = cfg->if_freq;
  p.l1_if_step = cfg->l1_if_step;
  p.glo_zero = cfg->glonass_zero_channel;
  p.spc = cfg->dll_spacing;
  p.pdi_code = 0.001;
  gnsscorr_sgt_loop_coefs(cfg, &p.tau1, &p.tau2, &p.k1, &p.k2, &p.k3);
  // padded code rows [c(end) c c(1)] as fp64 sign masks (tracking.sci:171-174)
  const int rows = cfg->system == 1 ? 1 : 33;
  uint32_t* h = (uint32_t*)calloc((size_t)rows * kPadLen, sizeof(uint32_t));
  int8_t chips[kMaxCode];
  const int L = cfg->code_length;
  for (int r = 0; r < rows; r++) {
    if (cfg->system == 1) gnsscorr_st_code(chips);
    else if (r == 0) continue;
    else gnsscorr_ca_code(r, chips);
    uint32_t* row = h + (size_t)r * kPadLen;
    auto m = [](int8_t v) { return v < 0 ? 0x80000000u : 0u; };
    row[0] = m(chips[L - 1]);
    for (int i = 0; i < L; i++) row[1 + i] = m(chips[i]);
    row[L + 1] = m(chips[0]);
  }
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc(&c->d_codes, sizeof(uint32_t) * rows * kPadLen);
  if (e == hipSuccess)
    e = hipMemcpy(c->d_codes, h, sizeof(uint32_t) * rows * kPadLen, hipMemcpyHostToDevice);
  free(h);
  if (e != hipSuccess) {
    gnsscorr_set_error("gnsscorr_sgt_create: %s", hipGetErrorString(e));
    gnsscorr_sgt_destroy(c);
    return GNSSCORR_EDEVICE;
  }
  *out = c;
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_track_dev(gnsscorr_sgt_ctx* c, const int8_t* d_if, int64_t stride,
                                      int64_t n_samples, int n_ch, gnsscorr_sgt_chan* d_chan,
                                      int n_epochs, int closed_loop, gnsscorr_sgt_epoch* d_ep) {
  if (!c || !d_if || !d_chan || !d_ep || n_ch < 1 || n_epochs < 1 || n_samples < 0 ||
      stride < 0) {
    gnsscorr_set_error("gnsscorr_sgt_track_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  if (c->cfg.file_type == 2 && ((uintptr_t)d_if & 1)) {
    gnsscorr_set_error("gnsscorr_sgt_track_dev: IQ record must be 2-byte aligned");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  // many channels: one wave per channel (throughput); fewer: 256-thread
  // workgroups, which also give the lowest epoch latency for the 14-channel
  // config-4 receiver (measured 9.3 us vs 9.4 / 11.6 us at 512 / 1024 threads,
  // 14.9 us at 128); a handful of channels: 512.  GNSSCORR_SGT_THREADS
  // overrides (64 = wave mode, 128..1024).
  int T = n_ch >= 1024 ? 64 : (n_ch >= 8 ? 256 : 512);
  if (const char* ov = getenv("GNSSCORR_SGT_THREADS")) {
    const int v = atoi(ov);
    if (v == 64 || v == 128 || v == 256 || v == 512 || v == 1024) T = v;
  }
  dim3 grid(n_ch), block(T);
  const size_t tab = sgt_tab_bytes(c->p.code_length);
  // + the prefix columns of the chunked path (64- and 256-thread shapes)
  const size_t tab_pf = tab + (sgt_prefix(T) ? (size_t)(T / 64) * kPfWaveBytes : 0);
#define SGT_LAUNCH(FT, CL)                                                                     \
  do {                                                                                         \
    if (T == 64)                                                                               \
      hipLaunchKernelGGL((sgt_track_kernel<FT, CL, 64>), grid, block, tab_pf, c->stream, c->p,\
                         d_if, stride, n_samples, c->d_codes, d_chan, n_epochs, d_ep);         \
    else if (T <= 256)                                                                         \
      hipLaunchKernelGGL((sgt_track_kernel<FT, CL, 256>), grid, block, tab_pf, c->stream,     \
                         c->p,                                                                 \
                         d_if, stride, n_samples, c->d_codes, d_chan, n_epochs, d_ep);         \
    else                                                                                       \
      hipLaunchKernelGGL((sgt_track_kernel<FT, CL, 1024>), grid, block, tab, c->stream, c->p, \
                         d_if, stride, n_samples, c->d_codes, d_chan, n_epochs, d_ep);         \
  } while (0)
  if (c->cfg.file_type == 2) {
    if (closed_loop) SGT_LAUNCH(2, true);
    else SGT_LAUNCH(2, false);
  } else {
    if (closed_loop) SGT_LAUNCH(1, true);
    else SGT_LAUNCH(1, false);
  }
#undef SGT_LAUNCH
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_track(gnsscorr_sgt_ctx* c, const int8_t* d_if, int64_t stride,
                                  int64_t n_samples, int n_ch, gnsscorr_sgt_chan* h_chan,
                                  int n_epochs, int closed_loop, gnsscorr_sgt_epoch* h_ep) {
  if (!c || !h_chan || !h_ep || n_ch < 1 || n_epochs < 1) {
    gnsscorr_set_error("gnsscorr_sgt_track: bad arguments");
    return GNSSCORR_EINVAL;
  }
  for (int i = 0; i < n_ch; i++) {
    const int id = h_chan[i].code_id;
    if (c->cfg.system == 0 ? (id < 1 || id > 32) : (id < -7 || id > 6)) {
      gnsscorr_set_error("gnsscorr_sgt_track: channel %d: bad PRN/FCH %d", i, id);
      return GNSSCORR_EINVAL;
    }
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const size_t nc = (size_t)n_ch, ne = nc * (size_t)n_epochs;
  if (nc > c->chan_cap) {
    (void)hipFree(c->d_chan);
    c->d_chan = nullptr;
    HIP_TRY(hipMalloc(&c->d_chan, nc * sizeof(gnsscorr_sgt_chan)));
    c->chan_cap = nc;
  }
  if (ne > c->ep_cap) {
    (void)hipFree(c->d_ep);
    c->d_ep = nullptr;
    HIP_TRY(hipMalloc(&c->d_ep, ne * sizeof(gnsscorr_sgt_epoch)));
    c->ep_cap = ne;
  }
  HIP_TRY(hipMemcpyAsync(c->d_chan, h_chan, nc * sizeof(gnsscorr_sgt_chan),
                         hipMemcpyHostToDevice, c->stream));
  int rc = gnsscorr_sgt_track_dev(c, d_if, stride, n_samples, n_ch, c->d_chan, n_epochs,
                                  closed_loop, c->d_ep);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(h_chan, c->d_chan, nc * sizeof(gnsscorr_sgt_chan),
                         hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(h_ep, c->d_ep, ne * sizeof(gnsscorr_sgt_epoch), hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_sync(gnsscorr_sgt_ctx* c) {
  if (!c) return GNSSCORR_EINVAL;
  HIP_TRY(hipSetDevice(c->cfg.device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return GNSSCORR_OK;
}

extern "C" void* gnsscorr_sgt_stream(gnsscorr_sgt_ctx* c) { return c ? (void*)c->stream : nullptr; }

extern "C" int gnsscorr_sgt_replay_dev(gnsscorr_sgt_ctx* c, int n_ch, gnsscorr_sgt_chan* d_chan,
                                       int n_epochs, const double* d_sums,
                                       gnsscorr_sgt_epoch* d_ep) {
  if (!c || !d_chan || !d_sums || !d_ep || n_ch < 1 || n_epochs < 1) {
    gnsscorr_set_error("gnsscorr_sgt_replay_dev: bad arguments");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  hipLaunchKernelGGL(sgt_replay_kernel, dim3((n_ch + 63) / 64), dim3(64), 0, c->stream, c->p,
                     d_chan, n_ch, n_epochs, d_sums, d_ep);
  HIP_TRY(hipGetLastError());
  return GNSSCORR_OK;
}

extern "C" int gnsscorr_sgt_replay(gnsscorr_sgt_ctx* c, int n_ch, gnsscorr_sgt_chan* h_chan,
                                   int n_epochs, const double* h_sums, gnsscorr_sgt_epoch* h_ep) {
  if (!c || !h_chan || !h_sums || !h_ep || n_ch < 1 || n_epochs < 1) {
    gnsscorr_set_error("gnsscorr_sgt_replay: bad arguments");
    return GNSSCORR_EINVAL;
  }
  HIP_TRY(hipSetDevice(c->cfg.device));
  const size_t nc = (size_t)n_ch, ne = nc * (size_t)n_epochs;
  gnsscorr_sgt_chan* d_chan = nullptr;
  double* d_sums = nullptr;
  gnsscorr_sgt_epoch* d_ep = nullptr;
  hipError_t e = hipMalloc(&d_chan, nc * sizeof(gnsscorr_sgt_chan));
  if (e == hipSuccess) e = hipMalloc(&d_sums, ne * 6 * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&d_ep, ne * sizeof(gnsscorr_sgt_epoch));
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_chan, h_chan, nc * sizeof(gnsscorr_sgt_chan), hipMemcpyHostToDevice,
                       c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(d_sums, h_sums, ne * 6 * sizeof(double), hipMemcpyHostToDevice,
                       c->stream);
  int rc = GNSSCORR_OK;
  if (e == hipSuccess) rc = gnsscorr_sgt_replay_dev(c, n_ch, d_chan, n_epochs, d_sums, d_ep);
  if (e == hipSuccess && rc == GNSSCORR_OK)
    e = hipMemcpyAsync(h_chan, d_chan, nc * sizeof(gnsscorr_sgt_chan), hipMemcpyDeviceToHost,
                       c->stream);
  if (e == hipSuccess && rc == GNSSCORR_OK)
    e = hipMemcpyAsync(h_ep, d_ep, ne * sizeof(gnsscorr_sgt_epoch), hipMemcpyDeviceToHost,
                       c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(d_chan);
  (void)hipFree(d_sums);
  (void)hipFree(d_ep);
  if (e != hipSuccess) {
    gnsscorr_set_error("gnsscorr_sgt_replay: %s", hipGetErrorString(e));
    return GNSSCORR_EDEVICE;
  }
  return rc;
}
