// Round-4 experiment: why the headline launch (the production node fold, float, 8 ranks x 16 MiB,
// U 4 staggered) runs faster when bench.py rotates 3 buffer sets (768 MiB) than 4 or 6
// (tools/xcdmap.hip, profiles/r04/xcd/). The send buffers (only read) and the receive buffers
// (only written) rotate independently here: launch i reads send set i mod SS and writes receive
// set i mod RS. If the 3-set rotation is faster because the Infinity Cache still holds part of a
// receive set's lines when the set is written again (a dirty line overwritten in the cache is
// never written to HBM), the time follows RS; if it is address translation reach or the cache
// as a whole, it follows the total footprint.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -mllvm -amdgpu-kernarg-preload-count=16 tools/setsweep.hip -o tools/setsweep
// Run:   tools/setsweep [MiB per rank = 16] [rounds = 5] [launches = 48]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../ext_mpi_collectives_amd/csrc/fold_kernel.hpp"

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int R = 8, U = 4, ISSUE = 5, MAXSETS = 8;
constexpr long TILE = (long)EMAC_BLOCK * U;

int main(int argc, char **argv) {
  const long mib = argc > 1 ? atol(argv[1]) : 16;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5, launches = argc > 3 ? atoi(argv[3]) : 48;
  const long S = mib << 20, C = S / R, nvec = C / 16, tpb = nvec / TILE, ntiles = tpb * R;
  if (nvec % TILE) return 2;
  const unsigned grid = (unsigned)(ntiles < 8192 ? ntiles : 8192);
  std::vector<float *> sb(MAXSETS * R), rb(MAXSETS * R);
  for (int st = 0; st < MAXSETS; ++st)
    for (int r = 0; r < R; ++r) {  // as bench.py: each rank's send then receive buffer
      CHECK(hipMalloc(&sb[st * R + r], S));
      CHECK(hipMalloc(&rb[st * R + r], S));
      std::vector<float> hv(S / 4);
      unsigned long long x = 0x9E3779B97F4A7C15ull * (st * R + r + 1);
      for (auto &e : hv) {  // random integers: every fold order exact
        x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
        e = (float)((long)((x * 0x2545F4914F6CDD1Dull) >> 43) - (1L << 20));
      }
      CHECK(hipMemcpy(sb[st * R + r], hv.data(), S, hipMemcpyHostToDevice));
    }
  // a table per (send set, receive set): the plan's leaf order for '6;1 -8 8' (owner first)
  std::vector<emac_bucket *> tab(MAXSETS * MAXSETS);
  for (int a = 0; a < MAXSETS; ++a)
    for (int w = 0; w < MAXSETS; ++w) {
      std::vector<emac_bucket> h(R);
      for (int b = 0; b < R; ++b) {
        memset(&h[b], 0, sizeof(emac_bucket));
        for (int t = 0; t < R; ++t) {
          const int leaf = t == 0 ? b : t - 1 + (t - 1 >= b);
          h[b].src[t] = sb[a * R + leaf] + b * (C / 4);
          h[b].dst[t] = rb[w * R + t] + b * (C / 4);
        }
        h[b].nvec = nvec;
        h[b].tile0 = b * tpb;
        h[b].count = C / 4;
        h[b].ndst = R;
      }
      CHECK(hipMalloc(&tab[a * MAXSETS + w], sizeof(emac_bucket) * R));
      CHECK(hipMemcpy(tab[a * MAXSETS + w], h.data(), sizeof(emac_bucket) * R, hipMemcpyHostToDevice));
    }
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto launch = [&](int ss, int rs, int i) {
    hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, 0, R, ISSUE>), dim3(grid), dim3(EMAC_BLOCK), 0, s,
                       tab[(i % ss) * MAXSETS + (i % rs)], R, ntiles, tpb, 1, codes, (const unsigned *)nullptr, R);
  };
  const int combos[][2] = {{3, 3}, {4, 4}, {6, 6}, {6, 3}, {3, 6}, {8, 3}, {3, 8}, {2, 2}, {8, 8}, {6, 2}, {2, 6}};
  const int nc = sizeof(combos) / sizeof(combos[0]);
  std::vector<std::vector<double>> t(nc);
  printf("node fold 8 x %ld MiB (%ld MiB read + %ld MiB written per launch)\n", mib, R * mib, R * mib);
  for (int rd = 0; rd < rounds; ++rd)
    for (int c = 0; c < nc; ++c) {
      const int ss = combos[c][0], rs = combos[c][1];
      for (int i = 0; i < 2 * MAXSETS; ++i) launch(ss, rs, i);
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < launches; ++i) launch(ss, rs, i);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      t[c].push_back(ms * 1e3 / launches);
    }
  CHECK(hipGetLastError());
  for (int c = 0; c < nc; ++c) {
    std::vector<double> v = t[c];
    std::sort(v.begin(), v.end());
    const int ss = combos[c][0], rs = combos[c][1];
    printf("send sets %d (%4ld MiB) recv sets %d (%4ld MiB): median %7.2f us  min %7.2f  %.4f of 8 TB/s\n", ss,
           ss * R * mib, rs, rs * R * mib, v[v.size() / 2], v[0], 2.0 * R * S / v[v.size() / 2] / 8e6);
  }
  return 0;
}
