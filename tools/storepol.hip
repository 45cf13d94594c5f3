// Round-4 experiment: the store cache policy of the node fold. The fold's writes are what wait on
// DRAM credits ("The 256 MiB point"); every launch ends with the release that writes
// dirty L2 lines back. The production fold body (emac::load_fold<float, SUM, 8, U 4, linear,
// staggered issue>) with its 8 destination stores issued as buffer stores under each cache policy
// of gfx950 (aux bits: sc0 = 1, nt = 2, sc1 = 16), interleaved in one process, buffer sets rotated
// by read reuse (bench.py rotation_sets), at 16 and 256 MiB per rank:
//   global nt (the production store instruction), nt (2, its policy as a buffer store), plain (0), sc0 (1), sc0 nt (3), sc1 (16), sc1 nt (18),
//   sc0 sc1 (17, write-through to system scope), sc0 sc1 nt (19)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -mllvm -amdgpu-kernarg-preload-count=16 tools/storepol.hip -o tools/storepol
// Run:   tools/storepol [MiB per rank = 16] [rounds = 5] [launches = 30]
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

constexpr int R = 8, U = 4, ISSUE = 5;
constexpr long TILE = (long)EMAC_BLOCK * U;
typedef emac::Lane<float>::V V;

template <int AUX>
__global__ __launch_bounds__(EMAC_BLOCK) void k_store(const emac_bucket *__restrict__ bk, long tpb, long ntiles,
                                                      emac_codes codes) {
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bi = (int)((unsigned)tile / (unsigned)tpb);
    const long t = tile - (long)bi * tpb;
    const emac_bucket *b = bk + bi;
    V r[U];
    emac::load_fold<float, EMAC_SUM, R, U, 0, true, ISSUE>(b, t * TILE, 0, codes, r);
    if constexpr (AUX < 0) {  // the production stores: global_store_dwordx4 ... nt (emac::store_vec)
      typedef __attribute__((address_space(1))) V GV;
#pragma unroll
      for (int d = 0; d < R; ++d) {
        GV *dst = (GV *)b->dst[d] + t * TILE;
#pragma unroll
        for (int u = 0; u < U; ++u) emac::store_vec<V, ISSUE>(dst, threadIdx.x + (unsigned)(u * EMAC_BLOCK), r[u]);
      }
      continue;
    }
#pragma unroll
    for (int d = 0; d < R; ++d) {
      float *dst = (float *)b->dst[d] + t * TILE * 4;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; ++u)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(emac::U32x4, r[u]), rs,
                                               (threadIdx.x + (unsigned)(u * EMAC_BLOCK)) * 16u, 0, AUX);
    }
  }
}

int main(int argc, char **argv) {
  const long mib = argc > 1 ? atol(argv[1]) : 16;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5, launches = argc > 3 ? atoi(argv[3]) : 30;
  const long S = mib << 20, C = S / R, nvec = C / 16, tpb = nvec / TILE, ntiles = tpb * R;
  const int sets = 1 + (int)(((640L << 20) + R * S - 1) / (R * S));
  if (nvec % TILE) return 2;
  const unsigned grid = (unsigned)(ntiles < 8192 ? ntiles : 8192);
  std::vector<float *> sb(sets * R), rb(sets * R);
  std::vector<emac_bucket *> tab(sets);
  for (int st = 0; st < sets; ++st) {
    for (int r = 0; r < R; ++r) {
      CHECK(hipMalloc(&sb[st * R + r], S));
      CHECK(hipMalloc(&rb[st * R + r], S));
      const float v = (float)(r + st + 1);
      unsigned u;
      memcpy(&u, &v, 4);
      CHECK(hipMemsetD32((hipDeviceptr_t)sb[st * R + r], u, S / 4));
    }
    std::vector<emac_bucket> h(R);
    for (int b = 0; b < R; ++b) {
      memset(&h[b], 0, sizeof(emac_bucket));
      for (int t = 0; t < R; ++t) {
        const int leaf = t == 0 ? b : t - 1 + (t - 1 >= b);
        h[b].src[t] = sb[st * R + leaf] + b * (C / 4);
        h[b].dst[t] = rb[st * R + t] + b * (C / 4);
      }
      h[b].nvec = nvec;
      h[b].tile0 = b * tpb;
      h[b].count = C / 4;
      h[b].ndst = R;
    }
    CHECK(hipMalloc(&tab[st], sizeof(emac_bucket) * R));
    CHECK(hipMemcpy(tab[st], h.data(), sizeof(emac_bucket) * R, hipMemcpyHostToDevice));
  }
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  constexpr int NV = 9;
  const int aux[NV] = {-1, 2, 0, 1, 3, 16, 18, 17, 19};
  const char *names[NV] = {"global nt", "nt", "plain", "sc0", "sc0 nt", "sc1", "sc1 nt", "sc0 sc1", "sc0 sc1 nt"};
  auto launch = [&](int k, int st) {
    const dim3 g(grid), bl(EMAC_BLOCK);
    switch (aux[k]) {
      case -1: hipLaunchKernelGGL(k_store<-1>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 2: hipLaunchKernelGGL(k_store<2>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 0: hipLaunchKernelGGL(k_store<0>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 1: hipLaunchKernelGGL(k_store<1>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 3: hipLaunchKernelGGL(k_store<3>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 16: hipLaunchKernelGGL(k_store<16>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 18: hipLaunchKernelGGL(k_store<18>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      case 17: hipLaunchKernelGGL(k_store<17>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
      default: hipLaunchKernelGGL(k_store<19>, g, bl, 0, s, tab[st], tpb, ntiles, codes); break;
    }
  };
  std::vector<double> med[NV];
  printf("node fold 8 x %ld MiB, grid %u, %d sets\n", mib, grid, sets);
  for (int rd = 0; rd < rounds; ++rd)
    for (int k = 0; k < NV; ++k) {
      for (int i = 0; i < 2 * sets; ++i) launch(k, i % sets);
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < launches; ++i) launch(k, i % sets);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      med[k].push_back(ms * 1e3 / launches);
      // receive buffer k % 8 of set 0 holds 36 everywhere (small integers: any fold order)
      std::vector<float> hb(S / 4);
      CHECK(hipMemcpy(hb.data(), rb[k % R], S, hipMemcpyDeviceToHost));
      for (size_t e = 0; e < hb.size(); e += 1009)
        if (hb[e] != 36.0f) {
          printf("MISMATCH policy %s at %zu: %f\n", names[k], e, hb[e]);
          return 1;
        }
      CHECK(hipMemset(rb[k % R], 0, S));
    }
  for (int k = 0; k < NV; ++k) {
    std::vector<double> v = med[k];
    std::sort(v.begin(), v.end());
    printf("median %-11s %8.2f us  min %8.2f  %.4f of 8 TB/s\n", names[k], v[v.size() / 2], v[0],
           2.0 * R * S / v[v.size() / 2] / 8e6);
  }
  return 0;
}
