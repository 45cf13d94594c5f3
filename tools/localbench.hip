// localbench.hip -- the LOCAL fold of SURVEY.md 8(d) (R = 8 leaves of C bytes -> ONE destination,
// read-dominated: 8 bytes read per byte written), where the north star's ">= 80 % of HBM read
// bandwidth at 256 MiB" is defined (C = 32 MiB). One process, interleaved rounds, median per
// variant (cdna_hip_programming.md 5.4 rule 24):
//   prod_uU_iI   the production fold_kernel<float, SUM, 8, U, linear, fan-out 1, ISSUE I>
//   glds_uU      leaves staged by LDS-DMA (global_load_lds_dwordx4 nt), one tile per pass
//   glds_pipe    persistent, double-buffered LDS-DMA (tile i+1 in flight while tile i folds)
//   read_glds    read-only LDS-DMA stream over the same bytes (the measured read ceiling)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/localbench.hip -o tools/localbench
// Run:   tools/localbench [chunk MiB = 32] [rounds = 7] [launches per round = 10]
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

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) f4 G4;
typedef __attribute__((address_space(3))) f4 L4;
constexpr int R = 8;

struct Job {
  const f4 *src[R];
  f4 *dst;
  long nvec;
};

__device__ __forceinline__ void glds16(const f4 *g, L4 *l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                   (__attribute__((address_space(3))) void *)l, 16, 0, 2 /* nt */);
}

// one tile (256 * U vectors) per workgroup pass: every wave stages its U x 64 vectors of each leaf
// into its own LDS rows, waits, folds from LDS in leaf order, stores nt once
template <int U>
__global__ __launch_bounds__(256) void fold_glds(Job j, unsigned ntiles) {
  __shared__ f4 lds[R * U * 256];
  const unsigned wave = threadIdx.x >> 6;
  for (unsigned tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long base = (long)tile * 256 * U;
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u)
        glds16(j.src[s] + base + u * 256 + threadIdx.x, (L4 *)(lds + (s * U + u) * 256 + wave * 64));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 r = lds[u * 256 + threadIdx.x];
#pragma unroll
      for (int s = 1; s < R; ++s) r = r + lds[(s * U + u) * 256 + threadIdx.x];
      __builtin_nontemporal_store(r, (G4 *)j.dst + base + u * 256 + threadIdx.x);
    }
    __syncthreads();  // WAR on the LDS rows before the next pass's DMA
  }
}

// persistent, double-buffered: the DMA of the next tile is issued before the current one is
// waited for (R glds per lane per tile; waiting down to R outstanding retires the current tile)
__global__ __launch_bounds__(256) void fold_glds_pipe(Job j, unsigned ntiles) {
  __shared__ f4 lds[2][R * 256];
  unsigned tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto issue = [&](unsigned t, int buf) {
    const long base = (long)t * 256;
#pragma unroll
    for (int s = 0; s < R; ++s) glds16(j.src[s] + base + threadIdx.x, (L4 *)(lds[buf] + s * 256 + (threadIdx.x & ~63u)));
  };
  issue(tile, 0);
  int buf = 0;
  for (; tile < ntiles; tile += gridDim.x, buf ^= 1) {
    const unsigned next = tile + gridDim.x;
    if (next < ntiles) {
      issue(next, buf ^ 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    f4 r = lds[buf][threadIdx.x];
#pragma unroll
    for (int s = 1; s < R; ++s) r = r + lds[buf][s * 256 + threadIdx.x];
    __builtin_nontemporal_store(r, (G4 *)j.dst + (long)tile * 256 + threadIdx.x);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's reads of `buf` are done before it is re-filled
  }
}

__global__ __launch_bounds__(256) void read_glds(const f4 *__restrict__ a, long n, float *out) {
  __shared__ f4 lds[8 * 256];
  f4 acc = {0, 0, 0, 0};
  const long step = (long)gridDim.x * 256 * 8;
  for (long i0 = (long)blockIdx.x * 256 * 8; i0 < n; i0 += step) {
#pragma unroll
    for (int k = 0; k < 8; ++k) glds16(a + i0 + k * 256 + threadIdx.x, (L4 *)(lds + k * 256 + (threadIdx.x & ~63u)));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc += lds[threadIdx.x];
    __syncthreads();
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
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
  const long mib = argc > 1 ? atol(argv[1]) : 32;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 10;
  const long C = (mib << 20) / 16;  // vectors per leaf
  const int nsets = std::max<long>(2, (768L << 20) / ((R + 1) * (mib << 20)) + 1);
  std::vector<Job> jobs(nsets);
  std::vector<emac_bucket *> ebk(nsets);
  for (int st = 0; st < nsets; st++) {
    emac_bucket eb;
    memset(&eb, 0, sizeof(eb));
    for (int s = 0; s < R; s++) {
      f4 *p;
      CHECK(hipMalloc(&p, C * 16));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, p, C, 977u * st + s);
      jobs[st].src[s] = p;
      eb.src[s] = p;
    }
    CHECK(hipMalloc(&jobs[st].dst, C * 16));
    jobs[st].nvec = C;
    eb.dst[0] = jobs[st].dst;
    eb.ndst = 1;
    eb.count = C * 4;
    eb.nvec = C;
    CHECK(hipMalloc(&ebk[st], sizeof(eb)));
    CHECK(hipMemcpy(ebk[st], &eb, sizeof(eb), hipMemcpyHostToDevice));
  }
  f4 *ca;
  const long cn = (long)(R + 1) * C;  // the same bytes as one fold launch moves
  CHECK(hipMalloc(&ca, 2 * cn * 16));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, ca, 2 * cn, 4242u);
  float *dummy;
  CHECK(hipMalloc(&dummy, 64));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = R;
  CHECK(hipDeviceSynchronize());
  struct V {
    const char *name;
    int kind;
    std::vector<float> us;
  };
  std::vector<V> vs = {{"prod_u1_i1", 11, {}}, {"prod_u2_i1", 21, {}}, {"prod_u2_i0", 20, {}}, {"prod_u2_i5", 25, {}},
                       {"prod_u4_i1", 41, {}}, {"prod_u4_i0", 40, {}}, {"prod_u4_i5", 45, {}}, {"prod_u4_i3", 43, {}},
                       {"prod_u8_i1", 81, {}}, {"prod_u8_i0", 80, {}}, {"glds_u2", 102, {}},
                       {"prod_u4_g2048", 241, {}}, {"prod_u4_g1024", 341, {}}, {"prod_u8_g512", 381, {}},
                       {"prod_u8_g768", 481, {}}, {"read_glds", 120, {}}};
  if (getenv("LOCALBENCH_ALL"))
    vs.insert(vs.end() - 1, {{"glds_u1", 101, {}}, {"glds_u4", 104, {}}, {"glds_pipe", 110, {}}});
  auto run = [&](int kind, int set, int i) {
    if (kind >= 200) {  // grid-capped variants: grid = cap, grid-stride over the tiles
      const int U = (kind % 100) / 10;
      const long ntiles = C / (256L * U);
      const unsigned cap = kind / 100 == 2 ? 2048 : kind / 100 == 3 ? (U == 8 ? 512 : 1024) : 768;
      const dim3 g((unsigned)std::min<long>(ntiles, cap));
      if (U == 4)
        hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, false, 1, 1>), g, dim3(256), 0, s, ebk[set], 1, ntiles, ntiles, 1, codes, (const unsigned *)nullptr, R);
      else
        hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 8, false, 1, 1>), g, dim3(256), 0, s, ebk[set], 1, ntiles, ntiles, 1, codes, (const unsigned *)nullptr, R);
      return;
    }
    if (kind < 100) {
      const int U = kind / 10;
      const long ntiles = C / (256L * U);
      const dim3 g((unsigned)std::min<long>(ntiles, 8192));
#define P(u, iss) \
  case u * 10 + iss: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, u, false, 1, iss>), g, dim3(256), 0, s, ebk[set], 1, ntiles, ntiles, 1, codes, (const unsigned *)nullptr, R); break;
      switch (kind) { P(1, 1) P(2, 1) P(2, 0) P(2, 5) P(4, 1) P(4, 0) P(4, 5) P(4, 3) P(8, 1) P(8, 0) }
#undef P
      return;
    }
    switch (kind) {
    case 101: hipLaunchKernelGGL(fold_glds<1>, dim3(std::min<long>(C / 256, 8192)), dim3(256), 0, s, jobs[set], (unsigned)(C / 256)); break;
    case 102: hipLaunchKernelGGL(fold_glds<2>, dim3(std::min<long>(C / 512, 8192)), dim3(256), 0, s, jobs[set], (unsigned)(C / 512)); break;
    case 104: hipLaunchKernelGGL(fold_glds<4>, dim3(std::min<long>(C / 1024, 8192)), dim3(256), 0, s, jobs[set], (unsigned)(C / 1024)); break;
    case 110: hipLaunchKernelGGL(fold_glds_pipe, dim3(1024), dim3(256), 0, s, jobs[set], (unsigned)(C / 256)); break;
    case 120: hipLaunchKernelGGL(read_glds, dim3(2048), dim3(256), 0, s, ca + (i & 1) * cn, cn, dummy); break;
    }
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int k = 0;
  for (auto &v : vs)
    for (int i = 0; i < 3; i++) run(v.kind, (k++) % nsets, i);
  CHECK(hipStreamSynchronize(s));
  for (int rd = 0; rd < rounds; rd++)
    for (auto &v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) run(v.kind, (k++) % nsets, i);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / per);
    }
  CHECK(hipGetLastError());
  const double bytes = (double)(R + 1) * C * 16;
  printf("local fold: %d leaves x %ld MiB -> 1, %d sets, %d rounds x %d launches (median us, GB/s of %.0f MB)\n", R, mib,
         nsets, rounds, per, bytes / 1e6);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-12s %9.2f us  %7.1f GB/s  (min %.2f max %.2f)\n", v.name, med, bytes / (med * 1e-6) / 1e9, v.us.front(),
           v.us.back());
  }
  return 0;
}
