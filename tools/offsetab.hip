// Round-4 experiment: does the relative placement of the ranks' buffers matter? The production
// node fold (emac::fold_kernel<float, SUM, 8, U 4, linear, fan-out 8, staggered issue>) on 8 ranks'
// send and receive buffers that start at rank r x STRIDE bytes into a larger allocation, for
// STRIDE = 0, 256 B, 4 KiB, 64 KiB, 1 MiB + 4 KiB: the 8 leaves of one tile then sit at
// different offsets modulo the memory's channel interleave. Interleaved in one process, buffer
// sets rotated by read reuse (bench.py rotation_sets); the data are small integers.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -mllvm -amdgpu-kernarg-preload-count=16 tools/offsetab.hip -o tools/offsetab
// Run:   tools/offsetab [MiB per rank = 16] [rounds = 5] [launches = 30]
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

constexpr int R = 8, U = 4, ISSUE = 5, NS = 5;
constexpr long TILE = (long)EMAC_BLOCK * U;
constexpr long STRIDES[NS] = {0, 256, 4096, 65536, (1 << 20) + 4096};

int main(int argc, char **argv) {
  const long mib = argc > 1 ? atol(argv[1]) : 16;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5, launches = argc > 3 ? atoi(argv[3]) : 30;
  const long S = mib << 20, C = S / R, nvec = C / 16, tpb = nvec / TILE, ntiles = tpb * R;
  const int sets = 1 + (int)(((640L << 20) + R * S - 1) / (R * S));
  if (nvec % TILE) return 2;
  const unsigned grid = (unsigned)(ntiles < 8192 ? ntiles : 8192);
  const long pad = STRIDES[NS - 1] * R;
  // per stride and set: one allocation holding the 8 send buffers, one the 8 receive buffers,
  // each buffer S + its rank's offset apart
  std::vector<emac_bucket *> tab(NS * sets);
  std::vector<void *> allocs;
  std::vector<float *> rb0(NS);
  for (int k = 0; k < NS; ++k)
    for (int st = 0; st < sets; ++st) {
      char *sa, *ra;
      CHECK(hipMalloc(&sa, R * S + pad));
      CHECK(hipMalloc(&ra, R * S + pad));
      allocs.push_back(sa);
      allocs.push_back(ra);
      float *sb[R], *rb[R];
      for (int r = 0; r < R; ++r) {
        sb[r] = (float *)(sa + r * (S + STRIDES[k]));
        rb[r] = (float *)(ra + r * (S + STRIDES[k]));
        const float v = (float)(r + st + 1);
        unsigned u;
        memcpy(&u, &v, 4);
        CHECK(hipMemsetD32((hipDeviceptr_t)sb[r], u, S / 4));
      }
      if (st == 0) rb0[k] = rb[0];
      std::vector<emac_bucket> h(R);
      for (int b = 0; b < R; ++b) {
        memset(&h[b], 0, sizeof(emac_bucket));
        for (int t = 0; t < R; ++t) {
          const int leaf = t == 0 ? b : t - 1 + (t - 1 >= b);
          h[b].src[t] = sb[leaf] + b * (C / 4);
          h[b].dst[t] = rb[t] + b * (C / 4);
        }
        h[b].nvec = nvec;
        h[b].tile0 = b * tpb;
        h[b].count = C / 4;
        h[b].ndst = R;
      }
      CHECK(hipMalloc(&tab[k * sets + st], sizeof(emac_bucket) * R));
      CHECK(hipMemcpy(tab[k * sets + st], h.data(), sizeof(emac_bucket) * R, hipMemcpyHostToDevice));
    }
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto launch = [&](int k, int st) {
    hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, 0, R, ISSUE>), dim3(grid), dim3(EMAC_BLOCK), 0, s,
                       tab[k * sets + st], R, ntiles, tpb, 1, codes, (const unsigned *)nullptr, R);
  };
  std::vector<double> med[NS];
  printf("node fold 8 x %ld MiB, grid %u, %d sets; rank r's buffers at r x (S + stride)\n", mib, grid, sets);
  for (int rd = 0; rd < rounds; ++rd)
    for (int k = 0; k < NS; ++k) {
      for (int i = 0; i < 2 * sets; ++i) launch(k, i % sets);
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < launches; ++i) launch(k, i % sets);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      med[k].push_back(ms * 1e3 / launches);
      std::vector<float> hb(S / 4);
      CHECK(hipMemcpy(hb.data(), rb0[k], S, hipMemcpyDeviceToHost));
      for (size_t e = 0; e < hb.size(); e += 1009)
        if (hb[e] != 36.0f) {
          printf("MISMATCH stride %ld at %zu: %f\n", STRIDES[k], e, hb[e]);
          return 1;
        }
      CHECK(hipMemset(rb0[k], 0, S));
    }
  for (int k = 0; k < NS; ++k) {
    std::vector<double> v = med[k];
    std::sort(v.begin(), v.end());
    printf("stride %8ld B: median %8.2f us  min %8.2f  %.4f of 8 TB/s\n", STRIDES[k], v[v.size() / 2], v[0],
           2.0 * R * S / v[v.size() / 2] / 8e6);
  }
  for (void *p : allocs) CHECK(hipFree(p));
  return 0;
}
