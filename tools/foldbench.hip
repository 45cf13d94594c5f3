// foldbench.hip -- variant sweep of the node-form fold (R = 8 leaves, fused 8-way fan-out) on one
// MI355X, interleaved rounds in one process (cdna_hip_programming.md 5.4 rule 24). Also times a
// float4 copy and a float4 read-reduce over the same byte volume as ceilings.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/foldbench.hip -o tools/foldbench \
//          -Lext_mpi_collectives_amd -lext_mpi_amd -Wl,-rpath,'$ORIGIN/../ext_mpi_collectives_amd'
// Run:   ./foldbench [MiB per rank = 16] [rounds = 7] [launches per round = 20]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ext_mpi_amd.h"
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
constexpr int R = 8;

struct Bucket {
  const f4 *src[R];
  f4 *dst[R];
  long nvec;
};

template <bool NT>
__device__ __forceinline__ f4 ld(const f4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4 *p, f4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// tile = BLOCK*U vectors of one bucket; grid-stride over tiles; bucket = tile / tiles_per_bucket
template <int BLOCK, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(BLOCK) void fold(const Bucket *__restrict__ bk, long tiles_per_bucket, long ntiles) {
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Bucket *b = bk + tile / tiles_per_bucket;
    const long v0 = (tile % tiles_per_bucket) * (long)BLOCK * U + threadIdx.x;
    f4 x[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < R; ++s) {
        long v = v0 + (long)u * BLOCK;
        x[u][s] = v < b->nvec ? ld<NTL>(b->src[s] + v) : f4{0, 0, 0, 0};
      }
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = x[u][0];
#pragma unroll
      for (int s = 1; s < R; ++s) r[u] = r[u] + x[u][s];
    }
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long v = v0 + (long)u * BLOCK;
        if (v < b->nvec) st<NTS>(b->dst[d] + v, r[u]);
      }
  }
}

// harness kernel with global (address space 1) accesses, pointers still read lazily
template <int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void fold_glob(const Bucket *__restrict__ bk, long tiles_per_bucket, long ntiles) {
  typedef __attribute__((address_space(1))) f4 G;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Bucket *b = bk + tile / tiles_per_bucket;
    const long v0 = (tile % tiles_per_bucket) * (long)BLOCK * U + threadIdx.x;
    f4 x[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < R; ++s) {
        long v = v0 + (long)u * BLOCK;
        x[u][s] = v < b->nvec ? __builtin_nontemporal_load((const G *)b->src[s] + v) : f4{0, 0, 0, 0};
      }
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = x[u][0];
#pragma unroll
      for (int s = 1; s < R; ++s) r[u] = r[u] + x[u][s];
    }
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        long v = v0 + (long)u * BLOCK;
        if (v < b->nvec) __builtin_nontemporal_store(r[u], (G *)b->dst[d] + v);
      }
  }
}

// hoisted pointers + global accesses, loads issued source-major with a wave-level stagger
// (s_sleep after each group of 4 loads) to test whether burst issue hurts
template <int BLOCK, int U, int STAGGER>
__global__ __launch_bounds__(BLOCK) void fold_hoist(const Bucket *__restrict__ bk, long tiles_per_bucket, long ntiles) {
  typedef __attribute__((address_space(1))) f4 G;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Bucket *b = bk + (unsigned)tile / (unsigned)tiles_per_bucket;
    const long base = (long)((unsigned)tile % (unsigned)tiles_per_bucket) * BLOCK * U;
    const G *sp[R];
    G *dp[R];
#pragma unroll
    for (int s = 0; s < R; ++s) sp[s] = (const G *)b->src[s] + base;
#pragma unroll
    for (int s = 0; s < R; ++s) dp[s] = (G *)b->dst[s] + base;
    f4 x[U][R];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 0; s < R; ++s) {
        x[u][s] = __builtin_nontemporal_load(sp[s] + threadIdx.x + u * BLOCK);
        if (STAGGER && (s & 3) == 3) __builtin_amdgcn_s_sleep(STAGGER);
      }
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = x[u][0];
#pragma unroll
      for (int s = 1; s < R; ++s) r[u] = r[u] + x[u][s];
    }
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dp[d] + threadIdx.x + u * BLOCK);
  }
}

template <int BLOCK, int U>
void launch_glob(const Bucket *b, long tpb, long ntiles, hipStream_t s, int grid_cap) {
  long g = std::min<long>(ntiles, grid_cap);
  hipLaunchKernelGGL((fold_glob<BLOCK, U>), dim3(g), dim3(BLOCK), 0, s, b, tpb, ntiles);
}
template <int BLOCK, int U, int ST>
void launch_hoist(const Bucket *b, long tpb, long ntiles, hipStream_t s, int grid_cap) {
  long g = std::min<long>(ntiles, grid_cap);
  hipLaunchKernelGGL((fold_hoist<BLOCK, U, ST>), dim3(g), dim3(BLOCK), 0, s, b, tpb, ntiles);
}

// destination-major variant: each lane stores its U vectors to one destination before the next
template <int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void fold_wide(const Bucket *__restrict__ bk, long tiles_per_bucket, long ntiles) {
  // each block handles a tile but issues the 8 source loads for U vectors up front, the adds
  // in a running chain (fewer live registers), stores per destination
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const Bucket *b = bk + tile / tiles_per_bucket;
    const long v0 = (tile % tiles_per_bucket) * (long)BLOCK * U + threadIdx.x;
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = b->src[0][v0 + (long)u * BLOCK];
#pragma unroll
    for (int s = 1; s < R; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) r[u] = r[u] + b->src[s][v0 + (long)u * BLOCK];
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
      for (int u = 0; u < U; ++u) b->dst[d][v0 + (long)u * BLOCK] = r[u];
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
      v[k] = (float)((x >> 40) & 0xFFFFFF) / 8388608.0f - 1.0f;  // uniform [-1, 1)
    }
    p[i] = v;
  }
}

__global__ void copy_k(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void read_k(const f4 *__restrict__ a, long n, float *out) {
  f4 acc = {0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) acc += a[i];
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

struct Variant {
  const char *name;
  void (*launch)(const Bucket *, long, long, hipStream_t, int);
  int tile_vecs;
  std::vector<float> us;
};

template <int BLOCK, int U, bool NTL, bool NTS>
void launch_fold(const Bucket *b, long tpb, long ntiles, hipStream_t s, int grid_cap) {
  long g = std::min<long>(ntiles, grid_cap);
  hipLaunchKernelGGL((fold<BLOCK, U, NTL, NTS>), dim3(g), dim3(BLOCK), 0, s, b, tpb, ntiles);
}
template <int BLOCK, int U>
void launch_wide(const Bucket *b, long tpb, long ntiles, hipStream_t s, int grid_cap) {
  long g = std::min<long>(ntiles, grid_cap);
  hipLaunchKernelGGL((fold_wide<BLOCK, U>), dim3(g), dim3(BLOCK), 0, s, b, tpb, ntiles);
}

int main(int argc, char **argv) {
  long mib = argc > 1 ? atol(argv[1]) : 16;
  int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 20;
  long S = mib << 20, nvec_rank = S / 16, C = nvec_rank / R;  // vectors per chunk
  int nsets = std::max<long>(2, (640L << 20) / (2 * R * S) + 1);
  std::vector<Bucket *> dbk(nsets);
  std::vector<emac_bucket *> ebk_rot(nsets), ebk_prod(nsets);
  std::vector<f4 *> bufs;
  std::vector<int> prod_handles;
  for (int st = 0; st < nsets; st++) {
    f4 *send[R], *recv[R];
    for (int r = 0; r < R; r++) {
      CHECK(hipMalloc(&send[r], S));
      CHECK(hipMalloc(&recv[r], S));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, send[r], S / 16, 977u * st + r);
      bufs.push_back(send[r]);
      bufs.push_back(recv[r]);
    }
    {  // the production path on these same buffers, through the C ABI
      const void *sp[R];
      void *rp[R];
      for (int r = 0; r < R; r++) {
        sp[r] = send[r];
        rp[r] = recv[r];
      }
      int h;
      if (ext_mpi_amd_node_allreduce_init(R, sp, rp, S / 4, EXT_MPI_AMD_FLOAT, EXT_MPI_AMD_SUM, "6;1 -8 8", &h)) {
        fprintf(stderr, "node init failed\n");
        return 1;
      }
      prod_handles.push_back(h);
    }
    Bucket hb[R];
    for (int c = 0; c < R; c++) {
      for (int t = 0; t < R; t++) hb[c].src[t] = send[(c + t) % R] + c * C;
      for (int d = 0; d < R; d++) hb[c].dst[d] = recv[d] + c * C;
      hb[c].nvec = C;
    }
    {  // production kernel template on harness-built descriptors: rotated and production leaf order
      emac_bucket eb[2][R];
      memset(eb, 0, sizeof(eb));
      for (int o = 0; o < 2; o++)
        for (int c = 0; c < R; c++) {
          for (int t = 0; t < R; t++) {
            int leaf = o == 0 ? (c + t) % R : (t == 0 ? c : (t <= c ? t - 1 : t));
            eb[o][c].src[t] = send[leaf] + c * C;
          }
          for (int d = 0; d < R; d++) eb[o][c].dst[d] = recv[d] + c * C;
          eb[o][c].count = C * 4;
          eb[o][c].nvec = C;
          eb[o][c].ndst = R;
          eb[o][c].tile0 = (long)c * (C / 512);
        }
      CHECK(hipMalloc(&ebk_rot[st], sizeof(eb[0])));
      CHECK(hipMalloc(&ebk_prod[st], sizeof(eb[1])));
      CHECK(hipMemcpy(ebk_rot[st], eb[0], sizeof(eb[0]), hipMemcpyHostToDevice));
      CHECK(hipMemcpy(ebk_prod[st], eb[1], sizeof(eb[1]), hipMemcpyHostToDevice));
    }
    CHECK(hipMalloc(&dbk[st], sizeof(hb)));
    CHECK(hipMemcpy(dbk[st], hb, sizeof(hb), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  for (int h : prod_handles) ext_mpi_amd_set_stream(h, s);
  std::vector<float> prod_us, tmpl_rot_us, tmpl_prod_us;
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = R;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct V {
    const char *name;
    void (*fn)(const Bucket *, long, long, hipStream_t, int);
    int tile;
    int grid_cap;
    std::vector<float> us;
  };
  std::vector<V> vs = {
      {"b256_u2 (r1 prod)", launch_fold<256, 2, false, false>, 512, 8192, {}},
      {"b256_u2_ntls", launch_fold<256, 2, true, true>, 512, 8192, {}},
      {"glob_u2", launch_glob<256, 2>, 512, 8192, {}},
      {"hoist_u2", launch_hoist<256, 2, 0>, 512, 8192, {}},
      {"hoist_u2_sleep1", launch_hoist<256, 2, 1>, 512, 8192, {}},
      {"hoist_u2_sleep4", launch_hoist<256, 2, 4>, 512, 8192, {}},
      {"hoist_u2_g1792", launch_hoist<256, 2, 0>, 512, 1792, {}},
      {"b256_u2_ntls_g1792", launch_fold<256, 2, true, true>, 512, 1792, {}},
      {"hoist_u4", launch_hoist<256, 4, 0>, 1024, 8192, {}},
      {"hoist_u1", launch_hoist<256, 1, 0>, 256, 8192, {}},
      {"b256_u4_ntls", launch_fold<256, 4, true, true>, 1024, 8192, {}},
      {"b512_u2_ntls", launch_fold<512, 2, true, true>, 1024, 8192, {}},
      {"b256_u2_ntls", launch_fold<256, 2, true, true>, 512, 8192, {}},
  };
  // copy / read ceilings over the same bytes per launch as the fold (2RS: R*S read + R*S write)
  f4 *ca, *cb;
  long cn = R * S / 16;
  CHECK(hipMalloc(&ca, R * S * 2));
  CHECK(hipMalloc(&cb, R * S * 2));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, ca, R * S * 2 / 16, 4242u);
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, cb, R * S * 2 / 16, 4243u);
  CHECK(hipDeviceSynchronize());
  float *dummy;
  CHECK(hipMalloc(&dummy, 64));
  std::vector<float> copy_us, read_us;
  // correctness: every variant must produce the prod variant's bytes
  std::vector<char> ref(C * 16), got(C * 16);
  for (auto &v : vs)
    if (!strncmp(v.name, "wide", 4) && C % v.tile) {
      fprintf(stderr, "chunk not a multiple of the wide tile\n");
      return 1;
    }
  for (size_t vi = 0; vi < vs.size(); vi++) {
    long tpb = (C + vs[vi].tile - 1) / vs[vi].tile;
    vs[vi].fn(dbk[0], tpb, tpb * R, s, vs[vi].grid_cap);
    CHECK(hipStreamSynchronize(s));
    Bucket hb;
    CHECK(hipMemcpy(&hb, dbk[0] + 3, sizeof(hb), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(vi ? got.data() : ref.data(), hb.dst[5], C * 16, hipMemcpyDeviceToHost));
    if (vi && memcmp(ref.data(), got.data(), C * 16)) printf("MISMATCH %s\n", vs[vi].name);
  }
  int k = 0;
  for (int rd = 0; rd < rounds; rd++) {
    for (auto &v : vs) {
      long tpb = (C + v.tile - 1) / v.tile;
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) v.fn(dbk[(k++) % nsets], tpb, tpb * R, s, v.grid_cap);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000 / per);
    }
    for (int o = 0; o < 2; o++) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) {
        emac::Launch L = {&codes, (o ? ebk_prod : ebk_rot)[(k++) % nsets], R, (long)R * (C / 512), C / 512, 1, nullptr, 0, s};
        emac::launch_one<float, EMAC_SUM, R, 2, false, R>(L);
      }
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      (o ? tmpl_prod_us : tmpl_rot_us).push_back(ms * 1000 / per);
    }
    {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) ext_mpi_amd_start(prod_handles[(k++) % nsets]);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      prod_us.push_back(ms * 1000 / per);
    }
    for (int which = 0; which < 2; which++) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) {
        const f4 *src = ca + (i & 1) * cn;
        if (which == 0)
          hipLaunchKernelGGL(copy_k, dim3(8192), dim3(256), 0, s, src, cb + (i & 1) * cn, cn);
        else
          hipLaunchKernelGGL(read_k, dim3(8192), dim3(256), 0, s, (i & 1) ? cb : ca, 2 * cn, dummy);
      }
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      (which ? read_us : copy_us).push_back(ms * 1000 / per);
    }
  }
  auto med = [](std::vector<float> x) {
    std::sort(x.begin(), x.end());
    return x[x.size() / 2];
  };
  auto mn = [](std::vector<float> x) { return *std::min_element(x.begin(), x.end()); };
  double bytes = 2.0 * R * S;
  printf("# %ld MiB per rank, R=%d, %d sets, %d rounds x %d launches; GB/s = 2*R*S / t\n", mib, R, nsets, rounds, per);
  for (auto &v : vs)
    printf("%-20s median %8.2f us  min %8.2f us  %7.1f GB/s (best %7.1f)\n", v.name, med(v.us), mn(v.us),
           bytes / med(v.us) / 1e3, bytes / mn(v.us) / 1e3);
  printf("%-20s median %8.2f us  min %8.2f us  %7.1f GB/s\n", "PRODUCTION C-ABI", med(prod_us), mn(prod_us),
         bytes / med(prod_us) / 1e3);
  printf("%-20s median %8.2f us  min %8.2f us  %7.1f GB/s\n", "prod tmpl, rot order", med(tmpl_rot_us),
         mn(tmpl_rot_us), bytes / med(tmpl_rot_us) / 1e3);
  printf("%-20s median %8.2f us  min %8.2f us  %7.1f GB/s\n", "prod tmpl, prod order", med(tmpl_prod_us),
         mn(tmpl_prod_us), bytes / med(tmpl_prod_us) / 1e3);
  printf("%-20s median %8.2f us  %7.1f GB/s (read+write of %.0f MiB)\n", "copy float4", med(copy_us),
         bytes / med(copy_us) / 1e3, R * S / 1048576.0);
  printf("%-20s median %8.2f us  %7.1f GB/s (read of %.0f MiB)\n", "read float4", med(read_us),
         bytes / med(read_us) / 1e3, 2.0 * R * S / 1048576.0);
  return 0;
}
