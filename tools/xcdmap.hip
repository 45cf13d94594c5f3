// Round-4 experiment: an XCD-aware tile order for the node fold. MI355X dispatches workgroup i to
// XCD i mod 8, and every XCD has its own L2 and its own share of the fabric, so with
// tile = blockIdx.x the 8 XCDs take consecutive tiles in turn. Variants of the production node
// fold (emac::fold_vectors<float, SUM, 8 leaves, U 4, linear, fan-out 8, staggered issue>, the
// schedule the tuner keeps for configs[1]), interleaved in one process, buffer sets rotated past
// the Infinity Cache:
//   rr      tile = blockIdx.x (production): consecutive tiles on consecutive XCDs
//   xcd     each XCD takes one contiguous eighth of the tiles (with 8 equal owner chunks: one
//           owner chunk per XCD)
//   xcd4    runs of 4 consecutive tiles per XCD, the runs dealt out in turn
// each under three leaf orders of the owner chunks: identity (leaf t = rank t), the plan's for
// '6;1 -8 8' (the owner first, then the others ascending: the production order), and rotated
// (leaf t = rank (b + t) mod 8). Inputs are small integers, so every order folds to the same bits.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -mllvm -amdgpu-kernarg-preload-count=16 tools/xcdmap.hip -o tools/xcdmap
// Run:   tools/xcdmap [MiB per rank = 16] [rounds = 5] [launches per round = 30] [data = 2] [buffer sets]
// A tenth variant, prod, launches the production emac::fold_kernel itself on the plan-order table.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
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

__device__ __forceinline__ void tile_at(const emac_bucket *bk, long tpb, long tile, const emac_codes &c) {
  const int bi = (int)((unsigned)tile / (unsigned)tpb);
  const long t = tile - (long)bi * tpb;
  emac::fold_vectors<float, EMAC_SUM, R, U, 0, R, true, ISSUE>(bk + bi, t * TILE, 0, c);
}

template <int MAP>
__global__ __launch_bounds__(EMAC_BLOCK) void k_map(const emac_bucket *__restrict__ bk, long tpb, long ntiles,
                                                    emac_codes codes) {
  const unsigned xcd = blockIdx.x & 7, j = blockIdx.x >> 3, gx = gridDim.x >> 3;
  const long per = ntiles >> 3;  // tiles per XCD (ntiles % 8 == 0, gridDim.x % 8 == 0: host-checked)
  if constexpr (MAP == 0) {
    for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) tile_at(bk, tpb, tile, codes);
  } else if constexpr (MAP == 1) {
    for (long tl = j; tl < per; tl += gx) tile_at(bk, tpb, (long)xcd * per + tl, codes);
  } else {
    for (long tl = j; tl < per; tl += gx) tile_at(bk, tpb, ((tl >> 2) * 8 + xcd) * 4 + (tl & 3), codes);
  }
}

int main(int argc, char **argv) {
  const long mib = argc > 1 ? atol(argv[1]) : 16;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5, launches = argc > 3 ? atoi(argv[3]) : 30;
  const int data = argc > 4 ? atoi(argv[4]) : 2;  // 0 small integers, 1 one value near 1 per buffer, 2 random
  const long S = mib << 20, C = S / R, nvec = C / 16, tpb = nvec / TILE, ntiles = tpb * R;
  const int sets_dflt = (int)((640L << 20) / (2 * R * S) + 2 > 2 ? (640L << 20) / (2 * R * S) + 2 : 2);
  const int sets = argc > 5 ? atoi(argv[5]) : sets_dflt;
  if (nvec % TILE || ntiles % 8 || (ntiles / 8) % 4) {
    fprintf(stderr, "shape not whole tiles\n");
    return 2;
  }
  const unsigned grid = (unsigned)(ntiles < 8192 ? ntiles : 8192);
  std::vector<float *> sb(sets * R), rb(sets * R);
  std::vector<std::vector<float>> hs(sets * R);
  // leaf order of bucket (owner chunk) b: 0 identity, 1 the plan's for '6;1 -8 8' (owner first,
  // then the others ascending, plan.c), 2 rotated ((b + t) mod 8)
  std::vector<emac_bucket *> tabs(3 * sets);
  for (int st = 0; st < sets; ++st) {
    for (int r = 0; r < R; ++r) {
      CHECK(hipMalloc(&sb[st * R + r], S));
      CHECK(hipMalloc(&rb[st * R + r], S));
      if (data == 2) {  // random integers in [-2^20, 2^20): varied bits, every fold order exact
        std::vector<float> &hv = hs[st * R + r];
        hv.resize(S / 4);
        unsigned long long x = 0x9E3779B97F4A7C15ull * (st * R + r + 1);
        for (auto &e : hv) {
          x ^= x >> 12, x ^= x << 25, x ^= x >> 27;
          e = (float)((long)((x * 0x2545F4914F6CDD1Dull) >> 43) - (1L << 20));
        }
        CHECK(hipMemcpy(sb[st * R + r], hv.data(), S, hipMemcpyHostToDevice));
      } else {  // one value per buffer: small integers, or 1 + (r + st) / 128
        const float v = data == 0 ? (float)(r + st + 1) : 1.0f + (float)(r + st) / 128.0f;
        unsigned u;
        memcpy(&u, &v, 4);
        CHECK(hipMemsetD32((hipDeviceptr_t)sb[st * R + r], u, S / 4));
      }
    }
    for (int order = 0; order < 3; ++order) {
      std::vector<emac_bucket> h(R);
      for (int b = 0; b < R; ++b) {
        memset(&h[b], 0, sizeof(emac_bucket));
        for (int t = 0; t < R; ++t) {
          const int leaf = order == 0 ? t : order == 1 ? (t == 0 ? b : t - 1 + (t - 1 >= b)) : (b + t) % R;
          h[b].src[t] = sb[st * R + leaf] + b * (C / 4);
          h[b].dst[t] = rb[st * R + t] + b * (C / 4);
        }
        h[b].nvec = nvec;
        h[b].tile0 = b * tpb;
        h[b].count = C / 4;
        h[b].ndst = R;
      }
      CHECK(hipMalloc(&tabs[order * sets + st], sizeof(emac_bucket) * R));
      CHECK(hipMemcpy(tabs[order * sets + st], h.data(), sizeof(emac_bucket) * R, hipMemcpyHostToDevice));
    }
  }
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto launch = [&](int map, int st0) {
    if (map == 9) {  // the production kernel, plan order
      hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, 0, R, ISSUE>), dim3(grid), dim3(EMAC_BLOCK), 0, s,
                         tabs[sets + st0], R, ntiles, tpb, 1, codes, (const unsigned *)nullptr, R);
      return;
    }
    const int st = (map / 3) * sets + st0;  // variant = order * 3 + tile map
    map %= 3;
    switch (map) {
      case 0: hipLaunchKernelGGL(k_map<0>, dim3(grid), dim3(EMAC_BLOCK), 0, s, tabs[st], tpb, ntiles, codes); break;
      case 1: hipLaunchKernelGGL(k_map<1>, dim3(grid), dim3(EMAC_BLOCK), 0, s, tabs[st], tpb, ntiles, codes); break;
      default: hipLaunchKernelGGL(k_map<2>, dim3(grid), dim3(EMAC_BLOCK), 0, s, tabs[st], tpb, ntiles, codes); break;
    }
  };
  // the expected value of element k of set st (data 0 and 2 sum exactly in any order; data 1 is
  // checked in the identity order's bits only where every order agrees: its partial sums are exact too)
  auto want = [&](int st, size_t k) {
    float acc = 0.f;
    for (int r = 0; r < R; ++r)
      acc += data == 2 ? hs[st * R + r][k] : data == 0 ? (float)(r + st + 1) : 1.0f + (float)(r + st) / 128.0f;
    return acc;
  };
  const char *names[10] = {"rr/ident", "xcd/ident", "xcd4/ident", "rr/plan", "xcd/plan", "xcd4/plan",
                           "rr/rot", "xcd/rot", "xcd4/rot", "prod"};
  std::vector<double> med[10];
  printf("node fold 8 x %ld MiB, %ld tiles, grid %u, %d sets, data %d\n", mib, ntiles, grid, sets, data);
  for (int rd = 0; rd < rounds; ++rd) {
    for (int map = 0; map < 10; ++map) {
      for (int i = 0; i < 2 * sets; ++i) launch(map, i % sets);
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < launches; ++i) launch(map, i % sets);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / launches;
      med[map].push_back(us);
      bool ok = true;
      std::vector<float> hbuf(S / 4);
      for (int st = 0; st < sets && ok; ++st) {
        const int r = (st * 3 + map) % R;  // a different receive buffer per variant
        CHECK(hipMemcpy(hbuf.data(), rb[st * R + r], S, hipMemcpyDeviceToHost));
        for (size_t k = 0; k < hbuf.size(); k += 997)
          if (hbuf[k] != want(st, k)) { ok = false; break; }
        if (hbuf.back() != want(st, hbuf.size() - 1)) ok = false;
        CHECK(hipMemset(rb[st * R + r], 0, S));
      }
      printf("round %d %-10s %8.2f us  %.4f of 8 TB/s  %s\n", rd, names[map], us, 2.0 * R * S / us / 8e6,
             ok ? "ok" : "MISMATCH");
      fflush(stdout);
      if (!ok) return 1;
    }
  }
  for (int map = 0; map < 10; ++map) {
    std::vector<double> v = med[map];
    std::sort(v.begin(), v.end());
    printf("median %-10s %8.2f us  %.4f of 8 TB/s\n", names[map], v[v.size() / 2], 2.0 * R * S / v[v.size() / 2] / 8e6);
  }
  return 0;
}
