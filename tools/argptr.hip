// Round-4 experiment: does the bucket descriptor's scalar load cost a
// configs[2]-sized launch anything measurable? The int node fold of configs[2] (8 ranks x 4 MiB,
// 8 owner chunks of 512 KiB, U 4 tiles of 16 KiB per leaf, fan-out 8, nontemporal loads and
// stores, one 16 KiB tile per workgroup) in four forms, interleaved, 10 buffer sets rotated past
// the Infinity Cache:
//   table  -- as fold_kernel: each workgroup reads its bucket's leaf and destination pointers
//             from a device descriptor table (one dependent scalar load before the first leaf load)
//   args   -- the 8 leaf base pointers as the first 16 argument dwords (preloaded into SGPRs at
//             wave launch), the destinations and the chunk stride as later arguments
//   tagged -- as args, the chunk stride (in tiles) carried in leaf pointer 0's top 16 bits, so
//             nothing the first loads need comes from memory
//   const  -- as args, the stride a compile-time constant (the bound of the idea)
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-kernarg-preload-count=16 tools/argptr.hip -o tools/argptr
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) v4 gv4;
constexpr int B = 256, U = 4, N = 8;
constexpr long TILE = (long)B * U;              // vectors per leaf per tile
constexpr long CHUNK_VEC = (512L << 10) / 16;   // one owner chunk, 16-byte vectors
constexpr long TPB = CHUNK_VEC / TILE;          // tiles per bucket (32)

struct Bucket {
  const v4 *src[16];
  long nvec, tile0;
  v4 *dst[16];
  long count, head, tail;
  int ndst, scalar;
};

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__device__ __forceinline__ void tile_body(const gv4 *const (&src)[N], gv4 *const (&dst)[N]) {
  v4 x[U][N];
#pragma unroll
  for (int k = 0; k < N * U; ++k) {
    const int s = k % N, u = k / N;
    x[u][s] = __builtin_nontemporal_load(src[s] + threadIdx.x + u * B);
  }
  v4 r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    r[u] = x[u][0];
#pragma unroll
    for (int s = 1; s < N; ++s) r[u] += x[u][s];
  }
#pragma unroll
  for (int d = 0; d < N; ++d)
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst[d] + threadIdx.x + u * B);
}

__global__ __launch_bounds__(B) void k_table(const Bucket *__restrict__ bk, long tpb, long ntiles) {
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bi = (int)((unsigned)tile / (unsigned)tpb);
    const long base = (tile - (long)bi * tpb) * TILE;
    const Bucket *b = bk + bi;
    const gv4 *src[N];
    gv4 *dst[N];
#pragma unroll
    for (int s = 0; s < N; ++s) src[s] = (const gv4 *)b->src[s] + base;
#pragma unroll
    for (int d = 0; d < N; ++d) dst[d] = (gv4 *)b->dst[d] + base;
    tile_body(src, dst);
  }
}

// MODE 0: stride argument; 1: stride in s0's top 16 bits (tiles); 2: compile-time stride
template <int MODE>
__global__ __launch_bounds__(B) void k_args(const v4 *s0, const v4 *s1, const v4 *s2, const v4 *s3, const v4 *s4,
                                            const v4 *s5, const v4 *s6, const v4 *s7, v4 *d0, v4 *d1, v4 *d2, v4 *d3,
                                            v4 *d4, v4 *d5, v4 *d6, v4 *d7, long stride_tiles) {
  long tpb;
  const v4 *p0 = s0;
  if constexpr (MODE == 1) {
    tpb = (long)((unsigned long)s0 >> 48);
    p0 = (const v4 *)((unsigned long)s0 & ((1UL << 48) - 1));
  } else if constexpr (MODE == 2) {
    tpb = TPB;
  } else {
    tpb = stride_tiles;
  }
  // grid (tiles per bucket, buckets): the tile's vector offset inside leaf s
  const long base = ((long)blockIdx.y * tpb + blockIdx.x) * TILE;
  const gv4 *src[N] = {(const gv4 *)p0 + base, (const gv4 *)s1 + base, (const gv4 *)s2 + base, (const gv4 *)s3 + base,
                       (const gv4 *)s4 + base, (const gv4 *)s5 + base, (const gv4 *)s6 + base, (const gv4 *)s7 + base};
  gv4 *dst[N] = {(gv4 *)d0 + base, (gv4 *)d1 + base, (gv4 *)d2 + base, (gv4 *)d3 + base,
                 (gv4 *)d4 + base, (gv4 *)d5 + base, (gv4 *)d6 + base, (gv4 *)d7 + base};
  tile_body(src, dst);
}

int main(int argc, char **argv) {
  const int sets = 10, reps = argc > 1 ? atoi(argv[1]) : 3, launches = 200;
  const size_t bytes = 8 * CHUNK_VEC * 16;  // 4 MiB per rank
  std::vector<v4 *> sb(sets * N), rb(sets * N);
  std::vector<Bucket *> tables(sets);
  for (int st = 0; st < sets; ++st) {
    for (int r = 0; r < N; ++r) {
      CK(hipMalloc(&sb[st * N + r], bytes));
      CK(hipMalloc(&rb[st * N + r], bytes));
      CK(hipMemsetD32((hipDeviceptr_t)sb[st * N + r], r + 1 + st, bytes / 4));
      if ((unsigned long)sb[st * N + r] >> 48) { fprintf(stderr, "pointer above 2^48\n"); return 2; }
    }
    Bucket h[N] = {};
    for (int b = 0; b < N; ++b) {
      for (int r = 0; r < N; ++r) {
        h[b].src[r] = sb[st * N + r] + b * CHUNK_VEC;
        h[b].dst[r] = rb[st * N + r] + b * CHUNK_VEC;
      }
      h[b].nvec = CHUNK_VEC;
      h[b].tile0 = b * TPB;
    }
    CK(hipMalloc(&tables[st], sizeof(h)));
    CK(hipMemcpy(tables[st], h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&](int mode, int st) {
    v4 *const *S = &sb[st * N];
    v4 *const *D = &rb[st * N];
    const dim3 g2((unsigned)TPB, N);
    if (mode == 0) {
      hipLaunchKernelGGL(k_table, dim3((unsigned)(TPB * N)), dim3(B), 0, s, tables[st], TPB, TPB * N);
    } else if (mode == 1) {
      hipLaunchKernelGGL(k_args<0>, g2, dim3(B), 0, s, S[0], S[1], S[2], S[3], S[4], S[5], S[6], S[7], D[0], D[1], D[2],
                         D[3], D[4], D[5], D[6], D[7], TPB);
    } else if (mode == 2) {
      const v4 *t0 = (const v4 *)((unsigned long)S[0] | ((unsigned long)TPB << 48));
      hipLaunchKernelGGL(k_args<1>, g2, dim3(B), 0, s, t0, S[1], S[2], S[3], S[4], S[5], S[6], S[7], D[0], D[1], D[2],
                         D[3], D[4], D[5], D[6], D[7], 0L);
    } else {
      hipLaunchKernelGGL(k_args<2>, g2, dim3(B), 0, s, S[0], S[1], S[2], S[3], S[4], S[5], S[6], S[7], D[0], D[1], D[2],
                         D[3], D[4], D[5], D[6], D[7], 0L);
    }
  };
  const char *names[4] = {"table", "args", "tagged", "const"};
  double sum[4] = {0, 0, 0, 0};
  for (int rep = 0; rep < reps; ++rep) {
    for (int mode = 0; mode < 4; ++mode) {
      for (int i = 0; i < 2 * sets; ++i) launch(mode, i % sets);
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < launches; ++i) launch(mode, i % sets);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / launches;
      sum[mode] += us;
      // every destination of every set holds sum over ranks of (r + 1 + st) = 36 + 8 st
      std::vector<int> h(bytes / 4);
      bool ok = true;
      for (int st = 0; st < sets && ok; ++st)
        for (int r = 0; r < N && ok; r += 7) {
          CK(hipMemcpy(h.data(), rb[st * N + r], bytes, hipMemcpyDeviceToHost));
          for (size_t k = 0; k < h.size(); k += 4093)
            if (h[k] != 36 + 8 * st) { ok = false; break; }
          if (h.back() != 36 + 8 * st) ok = false;
        }
      CK(hipMemset(rb[0], 0, bytes));
      printf("rep %d %-6s %.2f us/launch (%.4f of 8 TB/s) %s\n", rep, names[mode], us, 64.0 * (1 << 20) / us / 8e6,
             ok ? "ok" : "MISMATCH");
      fflush(stdout);
      if (!ok) return 1;
    }
  }
  for (int mode = 0; mode < 4; ++mode) printf("mean %-6s %.2f us\n", names[mode], sum[mode] / reps);
  return 0;
}
