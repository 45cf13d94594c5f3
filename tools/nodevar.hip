// nodevar.hip -- round-3 A/B harness: where does the NODE-form fold (8 ranks x S in one HBM,
// every owner chunk folded from 8 leaves and stored into all 8 receive buffers) lose against a
// 1:1 copy of the same bytes? Variants of the tile -> workgroup mapping and of the store order,
// each a small change to the production loop (fold_kernel.hpp fold_vectors, linear 8-leaf float
// fold, nontemporal loads / stores), interleaved rounds, median; buffer sets rotated beyond the
// 256 MiB Infinity Cache. The production fold_kernel (U 2 / U 4 burst) runs beside them.
//   MAP 0  grid-stride over tiles, bucket-major (production)
//   MAP 1  grid-stride, tile i of the launch = tile i / nb of bucket i % nb (the buckets interleaved)
//   MAP 2  blocked: workgroup g takes K consecutive tiles of one bucket, one after the other
//   SROT 0 destinations in rank order (production); 1 rotated by tile; 2 rotated by wave
//   grid   workgroups per launch (persistent grids of 256 / 512 / 768 or one per tile)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/nodevar.hip -o tools/nodevar
// Run:   tools/nodevar [chunk KiB = 2048] [rounds = 7] [launches per round = 10]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) f4 G4;
constexpr int R = 8;

struct Bk {
  const f4 *src[R];
  f4 *dst[R];
};

template <int U, int MAP, int SROT>
__global__ __launch_bounds__(256) void vfold(const Bk *__restrict__ bk, int nb, long tpb, int K) {
  constexpr long TILE = 256L * U;
  const long ntiles = tpb * nb;
  auto one = [&](int bi, long t) {
    const Bk *b = bk + bi;
    const G4 *src[R];
#pragma unroll
    for (int s = 0; s < R; ++s) src[s] = (const G4 *)b->src[s] + t * TILE;
    f4 x[U][R];
#pragma unroll
    for (int k = 0; k < R * U; ++k) {
      const int s = k / U, u = k % U;
      x[u][s] = __builtin_nontemporal_load(src[s] + threadIdx.x + u * 256);
    }
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 a = x[u][0];
#pragma unroll
      for (int s = 1; s < R; ++s) a = a + x[u][s];
      r[u] = a;
    }
    int rot = 0;
    if constexpr (SROT == 1) rot = (int)(t & (R - 1));
    if constexpr (SROT == 2) rot = (int)((threadIdx.x >> 6) * 2 & (R - 1));
#pragma unroll
    for (int dd = 0; dd < R; ++dd) {
      const int d = SROT ? ((dd + rot) & (R - 1)) : dd;
      G4 *dst = (G4 *)b->dst[d] + t * TILE;
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst + threadIdx.x + u * 256);
    }
  };
  if constexpr (MAP == 0) {
    for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) one((int)(tile / tpb), tile % tpb);
  } else if constexpr (MAP == 1) {
    for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) one((int)(tile % nb), tile / nb);
  } else {
    for (long blk = blockIdx.x; blk * K < ntiles; blk += gridDim.x)
      for (long tile = blk * K; tile < (blk + 1) * K && tile < ntiles; ++tile) one((int)(tile / tpb), tile % tpb);
  }
}

// the local fold of SURVEY.md 8(d): 8 leaves of one chunk -> 1 destination (one bucket)
template <int U>
__global__ __launch_bounds__(256) void lfold(const Bk *__restrict__ b, long ntiles) {
  constexpr long TILE = 256L * U;
  for (long t = blockIdx.x; t < ntiles; t += gridDim.x) {
    f4 x[U][R];
#pragma unroll
    for (int k = 0; k < R * U; ++k) {
      const int s = k / U, u = k % U;
      x[u][s] = __builtin_nontemporal_load((const G4 *)b->src[s] + t * TILE + threadIdx.x + u * 256);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 a = x[u][0];
#pragma unroll
      for (int s = 1; s < R; ++s) a = a + x[u][s];
      __builtin_nontemporal_store(a, (G4 *)b->dst[0] + t * TILE + threadIdx.x + u * 256);
    }
  }
}

// the local fold with its stores deferred: each workgroup folds KB consecutive tiles into LDS,
// then writes them out in one burst (fewer read/write turnarounds per DRAM page)
template <int U, int KB>
__global__ __launch_bounds__(256) void lfold_burst(const Bk *__restrict__ b, long ntiles) {
  constexpr long TILE = 256L * U;
  __shared__ f4 res[KB * U * 256];
  for (long g = blockIdx.x; g * KB < ntiles; g += gridDim.x) {
    for (int j = 0; j < KB; ++j) {
      const long t = g * KB + j;
      f4 x[U][R];
#pragma unroll
      for (int k = 0; k < R * U; ++k) {
        const int s = k / U, u = k % U;
        x[u][s] = __builtin_nontemporal_load((const G4 *)b->src[s] + t * TILE + threadIdx.x + u * 256);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        f4 a = x[u][0];
#pragma unroll
        for (int s = 1; s < R; ++s) a = a + x[u][s];
        res[(j * U + u) * 256 + threadIdx.x] = a;
      }
    }
#pragma unroll
    for (int q = 0; q < KB * U; ++q)
      __builtin_nontemporal_store(res[q * 256 + threadIdx.x], (G4 *)b->dst[0] + g * KB * TILE + q * 256 + threadIdx.x);
  }
}

// leaf-major groups: a workgroup's KB consecutive tiles are read leaf after leaf (each leaf's
// KB * U vectors back to back: KB * U KiB contiguous per wave) and accumulated in registers in the
// leaves' order (the linear fold's bits), then stored to every destination in one burst
template <int U, int KB, int D>
__global__ __launch_bounds__(256) void fold_leafmajor(const Bk *__restrict__ bk, int nb, long tpb) {
  constexpr long TILE = 256L * U;
  const long ngroups = tpb / KB * nb;
  for (long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int bi = (int)((unsigned)g / (unsigned)(tpb / KB));
    const long base = ((long)g - (long)bi * (tpb / KB)) * KB * TILE;
    const Bk *b = bk + bi;
    f4 acc[KB * U];
#pragma unroll
    for (int q = 0; q < KB * U; ++q) acc[q] = __builtin_nontemporal_load((const G4 *)b->src[0] + base + q * 256 + threadIdx.x);
#pragma unroll
    for (int s = 1; s < R; ++s) {
      f4 x[KB * U];
#pragma unroll
      for (int q = 0; q < KB * U; ++q) x[q] = __builtin_nontemporal_load((const G4 *)b->src[s] + base + q * 256 + threadIdx.x);
#pragma unroll
      for (int q = 0; q < KB * U; ++q) acc[q] = acc[q] + x[q];
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int q = 0; q < KB * U; ++q)
        __builtin_nontemporal_store(acc[q], (G4 *)b->dst[d] + base + q * 256 + threadIdx.x);
  }
}

// the node fold with its stores deferred: KB consecutive tiles of one bucket folded into LDS,
// then written to all R destinations in one burst
template <int U, int KB>
__global__ __launch_bounds__(256) void nfold_burst(const Bk *__restrict__ bk, int nb, long tpb) {
  constexpr long TILE = 256L * U;
  __shared__ f4 res[KB * U * 256];
  const long ngroups = tpb / KB * nb;
  for (long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int bi = (int)(g / (tpb / KB));
    const long t0 = (g % (tpb / KB)) * KB;
    const Bk *b = bk + bi;
    for (int j = 0; j < KB; ++j) {
      const long t = t0 + j;
      f4 x[U][R];
#pragma unroll
      for (int k = 0; k < R * U; ++k) {
        const int s = k / U, u = k % U;
        x[u][s] = __builtin_nontemporal_load((const G4 *)b->src[s] + t * TILE + threadIdx.x + u * 256);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        f4 a = x[u][0];
#pragma unroll
        for (int s = 1; s < R; ++s) a = a + x[u][s];
        res[(j * U + u) * 256 + threadIdx.x] = a;
      }
    }
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
      for (int q = 0; q < KB * U; ++q)
        __builtin_nontemporal_store(res[q * 256 + threadIdx.x], (G4 *)b->dst[d] + t0 * TILE + q * 256 + threadIdx.x);
  }
}

// pure write stream (nontemporal stores), K vectors per lane
template <int K>
__global__ __launch_bounds__(256) void write_k(f4 *__restrict__ b, long n, float v0) {
  const long step = (long)gridDim.x * 256 * K;
  const f4 v = {v0, v0, v0, v0};
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
#pragma unroll
    for (int k = 0; k < K; ++k) __builtin_nontemporal_store(v, (G4 *)b + i0 + k * 256);
  }
}

// a 1:1 copy in phases: each workgroup loads KB x 256 x U vectors into LDS, then stores them
template <int U, int KB>
__global__ __launch_bounds__(256) void copy_phased(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  __shared__ f4 res[KB * U * 256];
  constexpr long G = 256L * U * KB;
  for (long g0 = (long)blockIdx.x * G; g0 < n; g0 += (long)gridDim.x * G) {
#pragma unroll
    for (int q = 0; q < KB * U; ++q) res[q * 256 + threadIdx.x] = __builtin_nontemporal_load((const G4 *)a + g0 + q * 256 + threadIdx.x);
#pragma unroll
    for (int q = 0; q < KB * U; ++q) __builtin_nontemporal_store(res[q * 256 + threadIdx.x], (G4 *)b + g0 + q * 256 + threadIdx.x);
  }
}

// pure read streams: K vectors per lane in flight into VGPRs (nt), or LDS-DMA (global_load_lds nt)
template <int K>
__global__ __launch_bounds__(256) void read_vgpr(const f4 *__restrict__ a, long n, float *out) {
  f4 acc = {0, 0, 0, 0};
  const long step = (long)gridDim.x * 256 * K;
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
    f4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load((const G4 *)a + i0 + k * 256);
#pragma unroll
    for (int k = 0; k < K; ++k) acc += v[k];
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}
typedef __attribute__((address_space(3))) f4 L4;
__global__ __launch_bounds__(256) void read_glds(const f4 *__restrict__ a, long n, float *out) {
  __shared__ f4 lds[8 * 256];
  f4 acc = {0, 0, 0, 0};
  const long step = (long)gridDim.x * 256 * 8;
  for (long i0 = (long)blockIdx.x * 256 * 8; i0 < n; i0 += step) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(a + i0 + k * 256 + threadIdx.x),
                                       (__attribute__((address_space(3))) void *)(lds + k * 256 + (threadIdx.x & ~63u)), 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc += lds[threadIdx.x];
    __syncthreads();
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

template <int K, bool NT>
__global__ __launch_bounds__(256) void copy_k(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  const long step = (long)gridDim.x * 256 * K;
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
    f4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load((const G4 *)a + i0 + k * 256);
#pragma unroll
    for (int k = 0; k < K; ++k) __builtin_nontemporal_store(v[k], (G4 *)b + i0 + k * 256);
  }
}

__global__ void fill_random(f4 *p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned long x = (unsigned long)i * 0x9E3779B97F4A7C15ul + seed * 0xD1B54A32D192ED03ul;
    f4 v;
    for (int k = 0; k < 4; k++) {
      x ^= x >> 31;
      x *= 0xBF58476D1CE4E5B9ul;
      x ^= x >> 29;
      v[k] = (float)((x >> 40) & 0xFFFFFF) / 8388608.0f - 1.0f;
    }
    p[i] = v;
  }
}

int main(int argc, char **argv) {
  const long kib = argc > 1 ? atol(argv[1]) : 2048;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 10;
  const long C = (kib << 10) / 16;  // vectors per chunk (bucket)
  const long S = R * C;             // vectors per rank's message
  const long set_bytes = 2L * R * S * 16;
  const int nsets = (int)std::max<long>(2, (1024L << 20) / set_bytes + 1);
  std::vector<emac_bucket *> dprod(nsets), dplocal(nsets);
  std::vector<Bk *> dvar(nsets), dloc(nsets);
  float *dummy;
  CHECK(hipMalloc(&dummy, 64));
  std::vector<f4 *> sends(nsets * R), recvs(nsets * R);
  for (int st = 0; st < nsets; st++) {
    std::vector<emac_bucket> bk(R);
    std::vector<Bk> vb(R);
    for (int r = 0; r < R; r++) {
      CHECK(hipMalloc(&sends[st * R + r], S * 16));
      CHECK(hipMalloc(&recvs[st * R + r], S * 16));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, sends[st * R + r], S, 977u * st + r);
    }
    for (int c = 0; c < R; c++) {
      memset(&bk[c], 0, sizeof(emac_bucket));
      for (int t = 0; t < R; t++) vb[c].src[t] = sends[st * R + t] + c * C, bk[c].src[t] = (void *)vb[c].src[t];
      for (int r = 0; r < R; r++) vb[c].dst[r] = recvs[st * R + r] + c * C, bk[c].dst[r] = vb[c].dst[r];
      bk[c].ndst = R;
      bk[c].count = C * 4;
      bk[c].nvec = C;
    }
    CHECK(hipMalloc(&dprod[st], sizeof(emac_bucket) * R));
    CHECK(hipMemcpy(dprod[st], bk.data(), sizeof(emac_bucket) * R, hipMemcpyHostToDevice));
    {  // the production kernel's local fold: one bucket, every rank's whole send buffer -> rank 0's receive buffer
      emac_bucket pl;
      memset(&pl, 0, sizeof(pl));
      for (int t = 0; t < R; t++) pl.src[t] = sends[st * R + t];
      pl.dst[0] = recvs[st * R];
      pl.ndst = 1;
      pl.count = S * 4;
      pl.nvec = S;
      CHECK(hipMalloc(&dplocal[st], sizeof(emac_bucket)));
      CHECK(hipMemcpy(dplocal[st], &pl, sizeof(emac_bucket), hipMemcpyHostToDevice));
    }
    Bk lb;  // the local fold: every rank's whole send buffer (8 leaves of S) -> rank 0's receive buffer
    for (int t = 0; t < R; t++) lb.src[t] = sends[st * R + t];
    for (int r = 0; r < R; r++) lb.dst[r] = recvs[st * R];
    CHECK(hipMalloc(&dloc[st], sizeof(Bk)));
    CHECK(hipMemcpy(dloc[st], &lb, sizeof(Bk), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&dvar[st], sizeof(Bk) * R));
    CHECK(hipMemcpy(dvar[st], vb.data(), sizeof(Bk) * R, hipMemcpyHostToDevice));
  }
  const long copy_n = (long)R * S;
  f4 *ca;
  CHECK(hipMalloc(&ca, 4 * copy_n * 16));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, ca, 4 * copy_n, 4242u);
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = R;
  CHECK(hipDeviceSynchronize());
  struct V {
    std::string name;
    int id, grid;
    std::vector<float> us;
  };
  const long t2 = C / 512, t4 = C / 1024, lt1 = S / 256;
  std::vector<V> vs = {
      {"prod_u2", 0, 0, {}},           {"prod_u4", 1, 0, {}},
      {"v_u2_seq", 10, 0, {}},         {"v_u2_ilv", 11, 0, {}},         {"v_u2_srot_t", 12, 0, {}},
      {"v_u2_srot_w", 13, 0, {}},      {"v_u2_ilv_srot_t", 14, 0, {}},  {"v_u4_seq", 15, 0, {}},
      {"v_u4_srot_t", 16, 0, {}},      {"v_u2_g256", 10, 256, {}},     {"v_u2_g512", 10, 512, {}},
      {"v_u2_g768", 10, 768, {}},      {"v_u2_g1024", 10, 1024, {}},   {"v_u4_g256", 15, 256, {}},
      {"v_u4_g512", 15, 512, {}},      {"v_u2_blk4_g", 17, 0, {}},     {"v_u2_blk16_g", 18, 0, {}},
      {"v_u4_blk4_g", 19, 0, {}},      {"v_u4_ilv", 21, 0, {}},        {"v_u4_ilv_g256", 21, 256, {}},
      {"v_u4_ilv_g512", 21, 512, {}},  {"copy_k4_nt", 20, 0, {}},
      {"local_u1", 40, 0, {}},         {"local_u2", 41, 0, {}},        {"local_u4", 42, 0, {}},
      {"local_u2_g256", 41, 256, {}},  {"local_u2_g512", 41, 512, {}}, {"local_u4_g256", 42, 256, {}},
      {"local_u4_g512", 42, 512, {}},  {"local_u1_g1024", 40, 1024, {}}, {"local_u1_g2048", 40, 2048, {}},
      {"local_burst_u2_k4", 43, 0, {}}, {"local_burst_u2_k8", 44, 0, {}}, {"local_burst_u4_k4", 45, 0, {}},
      {"local_burst_u2_k8_g256", 44, 256, {}}, {"local_burst_u2_k4_g512", 43, 512, {}},
      {"local_burst_u2_k4_g256", 43, 256, {}}, {"local_burst_u2_k4_g768", 43, 768, {}},
      {"local_burst_u2_k8_g512", 44, 512, {}}, {"local_burst_u4_k4_g512", 45, 512, {}},
      {"node_burst_u2_k2", 46, 0, {}}, {"node_burst_u2_k4", 47, 0, {}}, {"node_burst_u2_k2_g512", 46, 512, {}},
      {"node_burst_u2_k4_g512", 47, 512, {}}, {"node_burst_u4_k2", 48, 0, {}}, {"node_burst_u2_k4_g256", 47, 256, {}},
      {"node_burst_u2_k8", 60, 0, {}}, {"node_burst_u4_k4", 61, 0, {}}, {"node_burst_u1_k8", 62, 0, {}},
      {"local_burst_u2_k16", 63, 0, {}}, {"local_burst_u4_k8", 64, 0, {}},
      {"write_k4", 53, 0, {}}, {"copy_phased_u2_k4", 54, 0, {}}, {"copy_phased_u2_k8", 55, 0, {}},
      {"copy_phased_u4_k4_g512", 56, 512, {}},
      {"plocal_u2", 70, 0, {}}, {"plocal_u4", 71, 0, {}}, {"plocal_u2_defer4", 72, 0, {}}, {"plocal_u4_defer4", 73, 0, {}},
      {"pnode_u2_defer4", 74, 0, {}}, {"pnode_u4_defer2", 75, 0, {}},
      {"node_leaf_u2_k4", 80, 0, {}}, {"node_leaf_u2_k8", 81, 0, {}}, {"node_leaf_u4_k4", 82, 0, {}},
      {"node_leaf_u1_k8", 86, 0, {}},
      {"local_leaf_u2_k4", 83, 0, {}}, {"local_leaf_u2_k8", 84, 0, {}}, {"local_leaf_u4_k4", 85, 0, {}},
      {"local_leaf_u1_k8", 87, 0, {}},
      {"read_vgpr_k4", 50, 0, {}},     {"read_vgpr_k8", 51, 0, {}},    {"read_glds", 52, 0, {}}};
  auto run = [&](const V &v, int i) {
    const int st = i % nsets;
    const long n2 = R * t2, n4 = R * t4;
    auto g = [&](long n) { return (unsigned)(v.grid ? v.grid : std::min<long>(n, 8192)); };
    f4 *ca0 = ca + (i & 1) * 2 * copy_n;
    switch (v.id) {
    case 0:
      hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, 0, R, 1>), dim3(g(n2)), dim3(256), 0, s, dprod[st], R,
                         n2, t2, 1, codes, (const unsigned *)nullptr, R);
      break;
    case 1:
      hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, 0, R, 1>), dim3(g(n4)), dim3(256), 0, s, dprod[st], R,
                         n4, t4, 1, codes, (const unsigned *)nullptr, R);
      break;
    case 10: hipLaunchKernelGGL((vfold<2, 0, 0>), dim3(g(n2)), dim3(256), 0, s, dvar[st], R, t2, 1); break;
    case 11: hipLaunchKernelGGL((vfold<2, 1, 0>), dim3(g(n2)), dim3(256), 0, s, dvar[st], R, t2, 1); break;
    case 12: hipLaunchKernelGGL((vfold<2, 0, 1>), dim3(g(n2)), dim3(256), 0, s, dvar[st], R, t2, 1); break;
    case 13: hipLaunchKernelGGL((vfold<2, 0, 2>), dim3(g(n2)), dim3(256), 0, s, dvar[st], R, t2, 1); break;
    case 14: hipLaunchKernelGGL((vfold<2, 1, 1>), dim3(g(n2)), dim3(256), 0, s, dvar[st], R, t2, 1); break;
    case 15: hipLaunchKernelGGL((vfold<4, 0, 0>), dim3(g(n4)), dim3(256), 0, s, dvar[st], R, t4, 1); break;
    case 16: hipLaunchKernelGGL((vfold<4, 0, 1>), dim3(g(n4)), dim3(256), 0, s, dvar[st], R, t4, 1); break;
    case 17: hipLaunchKernelGGL((vfold<2, 2, 0>), dim3((unsigned)((n2 + 3) / 4)), dim3(256), 0, s, dvar[st], R, t2, 4); break;
    case 18: hipLaunchKernelGGL((vfold<2, 2, 0>), dim3((unsigned)((n2 + 15) / 16)), dim3(256), 0, s, dvar[st], R, t2, 16); break;
    case 19: hipLaunchKernelGGL((vfold<4, 2, 0>), dim3((unsigned)((n4 + 3) / 4)), dim3(256), 0, s, dvar[st], R, t4, 4); break;
    case 20: hipLaunchKernelGGL((copy_k<4, true>), dim3(4096), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 21: hipLaunchKernelGGL((vfold<4, 1, 0>), dim3(g(n4)), dim3(256), 0, s, dvar[st], R, t4, 1); break;
    case 40: hipLaunchKernelGGL((lfold<1>), dim3(g(lt1)), dim3(256), 0, s, dloc[st], lt1); break;
    case 41: hipLaunchKernelGGL((lfold<2>), dim3(g(lt1 / 2)), dim3(256), 0, s, dloc[st], lt1 / 2); break;
    case 42: hipLaunchKernelGGL((lfold<4>), dim3(g(lt1 / 4)), dim3(256), 0, s, dloc[st], lt1 / 4); break;
    case 43: hipLaunchKernelGGL((lfold_burst<2, 4>), dim3(g(lt1 / 8)), dim3(256), 0, s, dloc[st], lt1 / 2); break;
    case 44: hipLaunchKernelGGL((lfold_burst<2, 8>), dim3(g(lt1 / 16)), dim3(256), 0, s, dloc[st], lt1 / 2); break;
    case 45: hipLaunchKernelGGL((lfold_burst<4, 4>), dim3(g(lt1 / 16)), dim3(256), 0, s, dloc[st], lt1 / 4); break;
    case 46: hipLaunchKernelGGL((nfold_burst<2, 2>), dim3(g(n2 / 2)), dim3(256), 0, s, dvar[st], R, t2); break;
    case 47: hipLaunchKernelGGL((nfold_burst<2, 4>), dim3(g(n2 / 4)), dim3(256), 0, s, dvar[st], R, t2); break;
    case 48: hipLaunchKernelGGL((nfold_burst<4, 2>), dim3(g(n4 / 2)), dim3(256), 0, s, dvar[st], R, t4); break;
    case 60: hipLaunchKernelGGL((nfold_burst<2, 8>), dim3(g(n2 / 8)), dim3(256), 0, s, dvar[st], R, t2); break;
    case 61: hipLaunchKernelGGL((nfold_burst<4, 4>), dim3(g(n4 / 4)), dim3(256), 0, s, dvar[st], R, t4); break;
    case 62: hipLaunchKernelGGL((nfold_burst<1, 8>), dim3(g(n2 * 2 / 8)), dim3(256), 0, s, dvar[st], R, t2 * 2); break;
    case 63: hipLaunchKernelGGL((lfold_burst<2, 16>), dim3(g(lt1 / 32)), dim3(256), 0, s, dloc[st], lt1 / 2); break;
    case 64: hipLaunchKernelGGL((lfold_burst<4, 8>), dim3(g(lt1 / 32)), dim3(256), 0, s, dloc[st], lt1 / 4); break;
    case 53: hipLaunchKernelGGL((write_k<4>), dim3(4096), dim3(256), 0, s, ca0 + copy_n, copy_n, 1.0f); break;
    case 54: hipLaunchKernelGGL((copy_phased<2, 4>), dim3((unsigned)std::min<long>(copy_n / 2048, 1L << 20)), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 55: hipLaunchKernelGGL((copy_phased<2, 8>), dim3((unsigned)std::min<long>(copy_n / 4096, 1L << 20)), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 56: hipLaunchKernelGGL((copy_phased<4, 4>), dim3(512), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 70:
    case 71:
    case 72:
    case 73: {
      const int U = (v.id == 70 || v.id == 72) ? 2 : 4;
      const long nt = S / (256L * U), groups = v.id >= 72 ? (nt + 3) / 4 : nt;
      const unsigned grid = (unsigned)std::min<long>(groups, 8192);
      if (v.id == 70)
        hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, 0, 1, 1>), dim3(grid), dim3(256), 0, s, dplocal[st], 1, nt, nt, 1, codes, (const unsigned *)nullptr, R);
      else if (v.id == 71)
        hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, 0, 1, 1>), dim3(grid), dim3(256), 0, s, dplocal[st], 1, nt, nt, 1, codes, (const unsigned *)nullptr, R);
      else if (v.id == 72)
        hipLaunchKernelGGL((emac::fold_deferred_kernel<float, EMAC_SUM, R, 2, 0, 1, 1 | emac::defer(4), true>), dim3(grid), dim3(256), 0, s, dplocal[st], nt, groups, codes);
      else
        hipLaunchKernelGGL((emac::fold_deferred_kernel<float, EMAC_SUM, R, 4, 0, 1, 1 | emac::defer(4), true>), dim3(grid), dim3(256), 0, s, dplocal[st], nt, groups, codes);
      break;
    }
    case 74:
      hipLaunchKernelGGL((emac::fold_deferred_kernel<float, EMAC_SUM, R, 2, 0, R, 1 | emac::defer(4), true>), dim3((unsigned)std::min<long>(n2 / 4, 8192)), dim3(256), 0, s, dprod[st],
                         t2, n2 / 4, codes);
      break;
    case 75:
      hipLaunchKernelGGL((emac::fold_deferred_kernel<float, EMAC_SUM, R, 4, 0, R, 1 | emac::defer(2), true>), dim3((unsigned)std::min<long>(n4 / 2, 8192)), dim3(256), 0, s, dprod[st],
                         t4, n4 / 2, codes);
      break;
    case 80: hipLaunchKernelGGL((fold_leafmajor<2, 4, R>), dim3(g(n2 / 4)), dim3(256), 0, s, dvar[st], R, t2); break;
    case 81: hipLaunchKernelGGL((fold_leafmajor<2, 8, R>), dim3(g(n2 / 8)), dim3(256), 0, s, dvar[st], R, t2); break;
    case 82: hipLaunchKernelGGL((fold_leafmajor<4, 4, R>), dim3(g(n4 / 4)), dim3(256), 0, s, dvar[st], R, t4); break;
    case 86: hipLaunchKernelGGL((fold_leafmajor<1, 8, R>), dim3(g(2 * n2 / 8)), dim3(256), 0, s, dvar[st], R, 2 * t2); break;
    case 83: hipLaunchKernelGGL((fold_leafmajor<2, 4, 1>), dim3(g(lt1 / 8)), dim3(256), 0, s, dloc[st], 1, lt1 / 2); break;
    case 84: hipLaunchKernelGGL((fold_leafmajor<2, 8, 1>), dim3(g(lt1 / 16)), dim3(256), 0, s, dloc[st], 1, lt1 / 2); break;
    case 85: hipLaunchKernelGGL((fold_leafmajor<4, 4, 1>), dim3(g(lt1 / 16)), dim3(256), 0, s, dloc[st], 1, lt1 / 4); break;
    case 87: hipLaunchKernelGGL((fold_leafmajor<1, 8, 1>), dim3(g(lt1 / 8)), dim3(256), 0, s, dloc[st], 1, lt1); break;
    case 50: hipLaunchKernelGGL((read_vgpr<4>), dim3(4096), dim3(256), 0, s, ca0, 2 * copy_n, dummy); break;
    case 51: hipLaunchKernelGGL((read_vgpr<8>), dim3(2048), dim3(256), 0, s, ca0, 2 * copy_n, dummy); break;
    case 52: hipLaunchKernelGGL(read_glds, dim3(2048), dim3(256), 0, s, ca0, 2 * copy_n, dummy); break;
    }
  };
  {  // every fold variant stores the same bits into every receive buffer
    std::vector<float> want((size_t)S * 4), got((size_t)S * 4);
    run(vs[0], 0);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(want.data(), recvs[R - 1], S * 16, hipMemcpyDeviceToHost));
    for (const V &v : vs) {
      if (v.id == 20 || (v.id >= 50 && v.id < 60)) continue;
      for (int r = 0; r < R; r++) CHECK(hipMemset(recvs[r], 0, S * 16));
      run(v, 0);
      CHECK(hipStreamSynchronize(s));
      const bool loc = (v.id >= 40 && v.id < 46) || (v.id >= 63 && v.id < 74) || (v.id >= 83 && v.id <= 85) || v.id == 87;
      for (int r = 0; r < (loc ? 1 : R); r++) {  // the local folds write rank 0's buffer only
        CHECK(hipMemcpy(got.data(), recvs[r], S * 16, hipMemcpyDeviceToHost));
        if (memcmp(got.data(), want.data(), S * 16)) printf("MISMATCH %s rank %d\n", v.name.c_str(), r);
      }
    }
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; w++)
    for (const V &v : vs) run(v, w);
  CHECK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; r++)
    for (V &v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) run(v, i);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / per);
    }
  const double node_bytes = 2.0 * R * S * 16;
  printf("node fold variants: chunk %ld KiB (%ld KiB per rank, %.1f MiB per launch), %d sets, %d rounds x %d launches: "
         "median min max us\n", kib, kib * R, node_bytes / 1048576.0, nsets, rounds, per);
  for (V &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    const bool local = (v.id >= 40 && v.id < 46) || (v.id >= 63 && v.id < 74) || (v.id >= 83 && v.id <= 85) || v.id == 87, rd = v.id >= 50 && v.id < 60;
    const double bytes = v.id == 53 ? 1.0 * copy_n * 16 : rd ? 2.0 * copy_n * 16 : local ? (R + 1.0) * S * 16 : 2.0 * R * S * 16;
    printf("%-18s %9.2f %9.2f %9.2f  %6.3f TB/s  %.3f of 8\n", v.name.c_str(), med, v.us.front(), v.us.back(),
           bytes / med / 1e6, bytes / med / 1e6 / 8.0);
  }
  // the tuner's view (engine.c emac_tune): each launch alone between two timing events, the
  // stream synchronised after it, against the back-to-back figure above
  printf("isolated launches (events around each, synchronised): median min us\n");
  for (V &v : vs) {
    if (!(v.id == 0 || v.id == 1 || v.id == 74 || v.id == 75 || v.id == 80 || v.id == 86 || v.id == 72 || v.id == 83))
      continue;
    std::vector<float> iso;
    for (int r = 0; r < rounds; r++)
      for (int i = 0; i < per; i++) {
        CHECK(hipEventRecord(e0, s));
        run(v, i);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        iso.push_back(ms * 1000.f);
      }
    std::sort(iso.begin(), iso.end());
    printf("iso %-18s %9.2f %9.2f\n", v.name.c_str(), iso[iso.size() / 2], iso.front());
  }
  // back to back but with a timing event between launches (the tuner's round-robin in a Start
  // sequence enqueued without host waits)
  printf("events between back-to-back launches: median min us\n");
  for (V &v : vs) {
    if (!(v.id == 0 || v.id == 1 || v.id == 74 || v.id == 75 || v.id == 80 || v.id == 86 || v.id == 72 || v.id == 83))
      continue;
    std::vector<hipEvent_t> ev(per + 1);
    for (auto &e : ev) CHECK(hipEventCreate(&e));
    std::vector<float> b2b;
    for (int r = 0; r < rounds; r++) {
      CHECK(hipEventRecord(ev[0], s));
      for (int i = 0; i < per; i++) {
        run(v, i);
        CHECK(hipEventRecord(ev[i + 1], s));
      }
      CHECK(hipEventSynchronize(ev[per]));
      for (int i = 1; i < per; i++) {  // the first launch follows an idle stream
        float ms;
        CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
        b2b.push_back(ms * 1000.f);
      }
    }
    for (auto &e : ev) CHECK(hipEventDestroy(e));
    std::sort(b2b.begin(), b2b.end());
    printf("ev  %-18s %9.2f %9.2f\n", v.name.c_str(), b2b[b2b.size() / 2], b2b.front());
  }
  return 0;
}
