// tools/trk_stream_stamps.hip -- diagnostic build of osg_stream_kernel with
// s_memrealtime stamps (100 MHz) per wave (lane 0): 0 start, 1 call set up (the
// last call of the launch), 2 its first piece landed, 3 its pieces done, 5 end
// of the launch (all K calls: the tool replays K = 4 calls in one launch).  Not part of the library; on the GPU box: bash tools/trk_stream_stamps.sh
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
__device__ unsigned long long* g_stamps;
#define STREAM_PSTAMP(i)                                                          \
  do {                                                                            \
    if ((threadIdx.x & 63) == 0) {                                                \
      unsigned long long _t;                                                      \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory"); \
      g_stamps[((size_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * 8 + (i)] = _t; \
    }                                                                             \
  } while (0)
#include "../gnss-sdr.ru_amd/csrc/track.hip"

int main(int argc, char** argv) {
  const bool cs1 = argc > 2 && argv[2][0] == 'c';   // "cs1": one stream per channel
  const int C = argc > 1 ? atoi(argv[1]) : 3072, NS = 16368, RX = cs1 ? C : (C + 11) / 12, K = 4;
  const int wpc = 1;
  gnsscorr_track_cfg cfg = {};
  cfg.n_channels = C;
  cfg.max_nsamp = NS;
  cfg.samp_rate = 16.368e6;
  cfg.iq = 1;
  gnsscorr_track_ctx* ctx;
  if (gnsscorr_track_create(&ctx, &cfg)) { printf("create failed\n"); return 1; }
  std::vector<int8_t> hif((size_t)RX * K * NS * 2);
  srand(3);
  for (auto& v : hif) v = (int8_t)((rand() & 3) * 2 - 3);
  std::vector<gnsscorr_nco_cmd> cmd((size_t)K * C);
  for (int k = 0; k < K * C; k++) {
    gnsscorr_nco_cmd& m = cmd[k];
    memset(&m, 0, sizeof m);
    m.prn = 1 + (k % C) % 32;
    m.stream = cs1 ? (k % C) : (k % C) / 12;
    m.carrier_incr = 635008600u + (uint32_t)((rand() % 524000) - 262000) * 20u;
    m.code_incr = 6710886u * 40u + (uint32_t)(rand() % 20) - 10u;
    m.epoch_load = -1;
  }
  int8_t* d_if; gnsscorr_nco_cmd* d_c; gnsscorr_track_result* d_r; unsigned long long* d_st;
  const int W = (C + kStreamCh - 1) / kStreamCh, NW = kStreamCh * wpc;
  (void)hipMalloc(&d_if, hif.size());
  (void)hipMalloc(&d_c, cmd.size() * sizeof(gnsscorr_nco_cmd));
  (void)hipMalloc(&d_r, cmd.size() * sizeof(gnsscorr_track_result));
  (void)hipMalloc(&d_st, (size_t)W * NW * 8 * 8);
  (void)hipMemset(d_st, 0, (size_t)W * NW * 8 * 8);
  (void)hipMemcpy(d_if, hif.data(), hif.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_c, cmd.data(), cmd.size() * sizeof(gnsscorr_nco_cmd), hipMemcpyHostToDevice);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_st, sizeof(d_st));
  const int64_t stride = (int64_t)K * NS;
  if (gnsscorr_track_replay_dev(ctx, d_if, stride, NS, K, d_c, d_r)) { printf("replay failed\n"); return 1; }
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> st((size_t)W * NW * 8);
  (void)hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);   // last call's stamps
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < W; b++) {
    t0 = std::min(t0, st[(size_t)b * NW * 8]);
    t1 = std::max(t1, st[(size_t)b * NW * 8 + 5]);
  }
  const char* nm[6] = {"start", "last call set up", "first piece landed", "pieces", "-", "to end"};
  printf("%s C=%d wpc=%d kernel span %.1f us\n", cs1 ? "cs1" : "rx12", C, wpc, (t1 - t0) / 100.0);
  for (int i = 0; i < 6; i++) {
    std::vector<double> v;
    for (int b = 0; b < W; b++)
      for (int wv = 0; wv < NW; wv++) {
        const unsigned long long* a = &st[((size_t)b * NW + wv) * 8];
        if (!a[0] || !a[i] || i == 4) continue;
        v.push_back(i == 0 ? (double)(a[0] - t0)
                           : (double)(a[i] - (i == 5 ? a[3] : a[i - 1])));
      }
    std::sort(v.begin(), v.end());
    if (v.empty()) continue;
    printf("  %-20s p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us\n", nm[i], v[v.size() / 10] / 100.0,
           v[v.size() / 2] / 100.0, v[v.size() * 9 / 10] / 100.0, v.back() / 100.0);
  }
  return 0;
}
