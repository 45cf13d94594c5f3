// Round-4 experiment: the load cache policy of the fold (tools/storepol.hip did the stores). The
// production fold body's leaf loads -- source-major, an s_sleep every 4 loads (ISSUE 5), U 4 --
// issued as 16-byte buffer loads under each gfx950 cache policy (aux bits sc0 = 1, nt = 2,
// sc1 = 16) against the production `global_load_dwordx4 ... nt`, the stores the production ones,
// interleaved in one process, buffer sets rotated by read reuse (bench.py rotation_sets):
//   node  the node fan-out, 8 ranks x MiB per rank (8 leaves -> 8 destinations per owner chunk)
//   local the local fold of SURVEY.md 8(d), 8 leaves of MiB -> 1 destination (read-bound)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -mllvm -amdgpu-kernarg-preload-count=16 tools/loadpol.hip -o tools/loadpol
// Run:   tools/loadpol node|local [MiB = 16] [rounds = 5] [launches = 30]
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

// LAUX < 0: the production loads (emac::load_fold); else buffer loads under policy LAUX
template <int LAUX, int D>
__global__ __launch_bounds__(EMAC_BLOCK) void k_load(const emac_bucket *__restrict__ bk, long tpb, long ntiles,
                                                     emac_codes codes) {
  typedef __attribute__((address_space(1))) V GV;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bi = (int)((unsigned)tile / (unsigned)tpb);
    const long t = tile - (long)bi * tpb;
    const emac_bucket *b = bk + bi;
    V r[U];
    if constexpr (LAUX < 0) {
      emac::load_fold<float, EMAC_SUM, R, U, 0, true, ISSUE>(b, t * TILE, 0, codes, r);
    } else {
      V x[U][R];
#pragma unroll
      for (int s = 0; s < R; ++s) {  // source-major, s_sleep 2 after every 4 loads (ISSUE 5)
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(b->src[s]), 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const unsigned off = (unsigned)((t * TILE + threadIdx.x + u * EMAC_BLOCK) * 16);
          x[u][s] = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, LAUX));
          if (((s * U + u) & 3) == 3 && s * U + u + 1 < R * U) __builtin_amdgcn_s_sleep(2);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        r[u] = x[u][0];
#pragma unroll
        for (int s = 1; s < R; ++s) r[u] = r[u] + x[u][s];
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      GV *dst = (GV *)b->dst[d] + t * TILE;
#pragma unroll
      for (int u = 0; u < U; ++u) emac::store_vec<V, ISSUE>(dst, threadIdx.x + (unsigned)(u * EMAC_BLOCK), r[u]);
    }
  }
}

int main(int argc, char **argv) {
  const bool local = argc > 1 && !strcmp(argv[1], "local");
  const long mib = argc > 2 ? atol(argv[2]) : (local ? 32 : 16);
  const int rounds = argc > 3 ? atoi(argv[3]) : 5, launches = argc > 4 ? atoi(argv[4]) : 30;
  // node: 8 buckets (owner chunks of S / 8) over 8 ranks' buffers of S; local: 1 bucket of S per leaf
  const long S = mib << 20, C = local ? S : S / R, nvec = C / 16, tpb = nvec / TILE, nb = local ? 1 : R,
             ntiles = tpb * nb;
  const long read_per_set = R * S;
  const int sets = 1 + (int)(((640L << 20) + read_per_set - 1) / read_per_set);
  if (nvec % TILE || (C / 16) * 16 != C) return 2;
  const unsigned grid = (unsigned)(ntiles < 8192 ? ntiles : 8192);
  const int ndst = local ? 1 : R;
  std::vector<float *> sb(sets * R), rb(sets * ndst);
  std::vector<emac_bucket *> tab(sets);
  for (int st = 0; st < sets; ++st) {
    for (int r = 0; r < R; ++r) {
      CHECK(hipMalloc(&sb[st * R + r], S));
      const float v = (float)(r + st + 1);
      unsigned u;
      memcpy(&u, &v, 4);
      CHECK(hipMemsetD32((hipDeviceptr_t)sb[st * R + r], u, S / 4));
    }
    for (int d = 0; d < ndst; ++d) CHECK(hipMalloc(&rb[st * ndst + d], S));
    std::vector<emac_bucket> h(nb);
    for (int b = 0; b < nb; ++b) {
      memset(&h[b], 0, sizeof(emac_bucket));
      for (int t = 0; t < R; ++t) {
        const int leaf = local ? t : (t == 0 ? b : t - 1 + (t - 1 >= b));
        h[b].src[t] = sb[st * R + leaf] + b * (C / 4);
      }
      for (int d = 0; d < ndst; ++d) h[b].dst[d] = rb[st * ndst + d] + b * (C / 4);
      h[b].nvec = nvec;
      h[b].tile0 = b * tpb;
      h[b].count = C / 4;
      h[b].ndst = ndst;
    }
    CHECK(hipMalloc(&tab[st], sizeof(emac_bucket) * nb));
    CHECK(hipMemcpy(tab[st], h.data(), sizeof(emac_bucket) * nb, hipMemcpyHostToDevice));
  }
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  constexpr int NV = 8;
  const char *names[NV] = {"global nt", "nt", "plain", "sc0", "sc0 nt", "sc1", "sc1 nt", "sc0 sc1 nt"};
  auto launch = [&](int k, int st) {
    const dim3 g(grid), bl(EMAC_BLOCK);
#define L(A)                                                                                       \
  do {                                                                                             \
    if (local)                                                                                     \
      hipLaunchKernelGGL((k_load<A, 1>), g, bl, 0, s, tab[st], tpb, ntiles, codes);                \
    else                                                                                           \
      hipLaunchKernelGGL((k_load<A, R>), g, bl, 0, s, tab[st], tpb, ntiles, codes);                \
  } while (0)
    switch (k) {
      case 0: L(-1); break;
      case 1: L(2); break;
      case 2: L(0); break;
      case 3: L(1); break;
      case 4: L(3); break;
      case 5: L(16); break;
      case 6: L(18); break;
      default: L(19); break;
    }
#undef L
  };
  std::vector<double> med[NV];
  const double bytes = local ? (R + 1.0) * S : 2.0 * R * S;
  printf("%s fold, 8 leaves x %ld MiB, grid %u, %d sets\n", local ? "local" : "node", mib, grid, sets);
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
      // destination 0 of set 0 holds 36 everywhere (small integers: any fold order)
      std::vector<float> hb(S / 4);
      CHECK(hipMemcpy(hb.data(), rb[0], S, hipMemcpyDeviceToHost));
      for (size_t e = 0; e < hb.size(); e += 1009)
        if (hb[e] != 36.0f) {
          printf("MISMATCH policy %s at %zu: %f\n", names[k], e, hb[e]);
          return 1;
        }
      CHECK(hipMemset(rb[0], 0, S));
    }
  for (int k = 0; k < NV; ++k) {
    std::vector<double> v = med[k];
    std::sort(v.begin(), v.end());
    printf("median %-11s %8.2f us  min %8.2f  %.4f of 8 TB/s\n", names[k], v[v.size() / 2], v[0],
           bytes / v[v.size() / 2] / 8e6);
  }
  return 0;
}
