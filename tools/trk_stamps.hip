// tools/trk_stamps.hip -- diagnostic build of osg_track_kernel with
// s_memrealtime stamps (100 MHz) at its phase boundaries, taken by thread 0
// and thread 192 (wave 3) of every workgroup.  Not part of the library; run
// on the GPU box: bash tools/trk_stamps.sh.  Phases: 0 start, 1 cmd/state read,
// 2 tables staged (barrier), 3 run done, 4 reduction barrier, 5 epilogue done.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
__device__ unsigned long long* g_stamps;
#define TRACK_PSTAMP(i)                                                          \
  do {                                                                           \
    if (threadIdx.x == 0 || threadIdx.x == 192) {                                \
      unsigned long long _t;                                                     \
      asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory"); \
      g_stamps[(blockIdx.x * 2 + (threadIdx.x ? 1 : 0)) * 8 + (i)] = _t;         \
    }                                                                            \
  } while (0)
#include "../gnss-sdr.ru_amd/csrc/track.hip"

int main(int argc, char** argv) {
  const bool cs1 = argc > 2 && argv[2][0] == 'c';   // "cs1": one stream per channel
  const int C = argc > 1 ? atoi(argv[1]) : 3072, NS = 16368, RX = cs1 ? C : (C + 11) / 12, K = 4;
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
  (void)hipMalloc(&d_if, hif.size());
  (void)hipMalloc(&d_c, cmd.size() * sizeof(gnsscorr_nco_cmd));
  (void)hipMalloc(&d_r, cmd.size() * sizeof(gnsscorr_track_result));
  (void)hipMalloc(&d_st, (size_t)C * 16 * 8);
  (void)hipMemcpy(d_if, hif.data(), hif.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(d_c, cmd.data(), cmd.size() * sizeof(gnsscorr_nco_cmd), hipMemcpyHostToDevice);
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_st, sizeof(d_st));
  const int64_t stride = (int64_t)K * NS;
  if (gnsscorr_track_replay_dev(ctx, d_if, stride, NS, K, d_c, d_r)) { printf("replay failed\n"); return 1; }
  (void)hipDeviceSynchronize();
  const int T = ((NS + 63) / 64 + 63) / 64 * 64, cpw = std::min(4, 1024 / T);
  const int W = (C + cpw - 1) / cpw;   // workgroups (the library's launch geometry)
  std::vector<unsigned long long> st((size_t)C * 16);
  (void)hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);   // last step's stamps
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < W; b++) { t0 = std::min(t0, st[b * 16 + 0]); t1 = std::max(t1, st[b * 16 + 5]); }
  double ph[6] = {0}, ph3w3 = 0;
  std::vector<double> starts, life;
  for (int b = 0; b < W; b++) {
    const unsigned long long* a = &st[b * 16];
    for (int i = 1; i < 6; i++) ph[i] += (double)(a[i] - a[i - 1]);
    ph3w3 += (double)(a[8 + 3] - a[8 + 2]);
    starts.push_back((double)(a[0] - t0));
    life.push_back((double)(a[5] - a[0]));
  }
  printf("%s C=%d kernel span %.1f us (stamp clock 100 MHz)\n", cs1 ? "cs1" : "rx12", C, (t1 - t0) / 100.0);
  const char* nm[6] = {"", "cmd/state", "tables+barrier", "run (wave 0)", "reduce+barrier", "epilogue"};
  for (int i = 1; i < 6; i++) printf("  %-16s %7.2f us\n", nm[i], ph[i] / W / 100.0);
  printf("  run (wave 3)     %7.2f us\n", ph3w3 / W / 100.0);
  std::sort(starts.begin(), starts.end());
  std::sort(life.begin(), life.end());
  printf("  WG lifetime p10/p50/p90 %.1f / %.1f / %.1f us\n", life[W / 10] / 100.0, life[W / 2] / 100.0,
         life[W * 9 / 10] / 100.0);
  for (int q = 1; q <= 8; q++) printf("  start of WG at %d/8: %.1f us\n", q, starts[(size_t)W * q / 8 - 1] / 100.0);
  return 0;
}
