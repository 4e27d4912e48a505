// tools/trk_clock_stamps.hip -- diagnostic build of osg_stream_kernel that stamps
// s_memtime (shader clock) and s_memrealtime (100 MHz) at each wave's start and
// end, so the in-kernel clock is Δmemtime / Δmemrealtime x 100 MHz
// (MI355X_MICROARCH.md, DVFS item 6).  The tool replays K = 10 calls per launch,
// L launches back to back (the bench's condition), and reports the last
// launch's per-wave clock and span for one stream per channel (cs1) or
// receivers of 12 channels (rx12).  Not part of the library; on the GPU box:
// bash tools/trk_clock_stamps.sh
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
__device__ unsigned long long* g_stamps;
#define STREAM_PSTAMP(i)                                                                   \
  do {                                                                                     \
    if ((i) == 0 || (i) == 5) {                                                            \
      if ((threadIdx.x & 63) == 0) {                                                       \
        unsigned long long _m, _r;                                                         \
        asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"            \
                     : "=s"(_m), "=s"(_r)::"memory");                                      \
        unsigned long long* _p =                                                           \
            g_stamps + ((size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * 4;  \
        _p[(i) == 0 ? 0 : 2] = _m;                                                         \
        _p[(i) == 0 ? 1 : 3] = _r;                                                         \
      }                                                                                    \
    }                                                                                      \
  } while (0)
#include "../gnss-sdr.ru_amd/csrc/track.hip"

int main(int argc, char** argv) {
  const int C = argc > 1 ? atoi(argv[1]) : 12288;
  const bool cs1 = argc > 2 && argv[2][0] == 'c';   // "cs1": one stream per channel
  const int L = argc > 3 ? atoi(argv[3]) : 30;      // launches back to back
  const int NS = 16368, RX = cs1 ? C : (C + 11) / 12, K = 10;
  gnsscorr_track_cfg cfg = {};
  cfg.n_channels = C;
  cfg.max_nsamp = NS;
  cfg.samp_rate = 16.368e6;
  cfg.iq = 1;
  gnsscorr_track_ctx* ctx;
  if (gnsscorr_track_create(&ctx, &cfg)) { printf("create failed\n"); return 1; }
  const size_t if_bytes = (size_t)RX * K * NS * 2;
  std::vector<gnsscorr_nco_cmd> cmd((size_t)K * C);
  srand(3);
  for (int k = 0; k < K * C; k++) {
    gnsscorr_nco_cmd& m = cmd[k];
    memset(&m, 0, sizeof m);
    m.prn = 1 + (k % C) % 32;
    m.stream = cs1 ? (k % C) : (k % C) / 12;
    m.carrier_incr = 635008600u + (uint32_t)((rand() % 524000) - 262000) * 20u;
    m.code_incr = 6710886u * 40u + (uint32_t)(rand() % 1600) - 800u;
    m.epoch_load = -1;
  }
  int8_t* d_if; gnsscorr_nco_cmd* d_c; gnsscorr_track_result* d_r; unsigned long long* d_st;
  const int W = (C + kStreamCh - 1) / kStreamCh, NW = kStreamCh;
  if (hipMalloc(&d_if, if_bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  (void)hipMalloc(&d_c, cmd.size() * sizeof(gnsscorr_nco_cmd));
  (void)hipMalloc(&d_r, cmd.size() * sizeof(gnsscorr_track_result));
  (void)hipMalloc(&d_st, (size_t)W * NW * 4 * 8);
  (void)hipMemset(d_st, 0, (size_t)W * NW * 4 * 8);
  if (gnsscorr_dev_fill_if2(0, d_if, if_bytes, 0x5EED000Bull)) { printf("fill failed\n"); return 1; }
  (void)hipMemcpy(d_c, cmd.data(), cmd.size() * sizeof(gnsscorr_nco_cmd), hipMemcpyHostToDevice);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_st, sizeof(d_st));
  const int64_t stride = (int64_t)K * NS;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int l = 0; l < L; l++) {
    if (l == L - 1) (void)hipEventRecord(e0, (hipStream_t)gnsscorr_track_stream(ctx));
    if (gnsscorr_track_replay_dev(ctx, d_if, stride, NS, K, d_c, d_r)) { printf("replay failed\n"); return 1; }
  }
  (void)hipEventRecord(e1, (hipStream_t)gnsscorr_track_stream(ctx));
  (void)hipDeviceSynchronize();
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> st((size_t)W * NW * 4);
  (void)hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);   // the last launch
  std::vector<double> ghz;
  unsigned long long r0 = ~0ull, r1 = 0;
  for (size_t w = 0; w < (size_t)W * NW; w++) {
    const unsigned long long* a = &st[w * 4];
    if (!a[0] || !a[2] || a[3] <= a[1]) continue;
    ghz.push_back((double)(a[2] - a[0]) / (double)(a[3] - a[1]) * 0.1);
    r0 = std::min(r0, a[1]);
    r1 = std::max(r1, a[3]);
  }
  std::sort(ghz.begin(), ghz.end());
  if (ghz.empty()) { printf("no stamps\n"); return 1; }
  printf("%s C=%d launch %.1f us (%.2f us per 3072 channel-ms), stamped span %.1f us, "
         "wave clock GHz p10 %.3f p50 %.3f p90 %.3f\n",
         cs1 ? "cs1" : "rx12", C, ms * 1e3, ms * 1e3 / K * 3072.0 / C, (r1 - r0) / 100.0,
         ghz[ghz.size() / 10], ghz[ghz.size() / 2], ghz[ghz.size() * 9 / 10]);
  return 0;
}
