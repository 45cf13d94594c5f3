// ldsbench.hip -- does LDS-DMA (global_load_lds_dwordx4, nt) lift the node-form fold above the
// register-load ceiling? One process, interleaved rounds (cdna_hip_programming.md 5.4 rule 24):
//   prod_u2 / prod_u4  the production fold_kernel template (R = 8 leaves, fan-out 8)
//   read_nt            read-only kernel, nt dwordx4 loads to VGPRs, same bytes as the fold moves
//   read_glds          read-only kernel, nt glds into LDS, same bytes
//   glds_u1 / glds_u2  fold with the leaves staged by glds (one tile per workgroup pass)
//   glds_pipe          persistent fold, glds double buffer (tile i+1 in flight while i folds)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/ldsbench.hip -o tools/ldsbench
// Run:   tools/ldsbench [MiB per rank = 16] [rounds = 7] [launches per round = 20]
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
constexpr int NT = 2;  // aux: nontemporal

struct Bucket {
  const f4 *src[R];
  f4 *dst[R];
  long nvec;
};

__device__ __forceinline__ void glds16(const f4 *g, L4 *l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                   (__attribute__((address_space(3))) void *)l, 16, 0, NT);
}

// one tile per workgroup pass: every wave stages its U x 64 vectors of each leaf into its own
// LDS rows, waits, folds from LDS, stores nt to the 8 destinations
template <int U>
__global__ __launch_bounds__(256) void fold_glds(const Bucket *__restrict__ bk, unsigned tpb, unsigned ntiles) {
  __shared__ f4 lds[R * U * 256];
  const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (unsigned tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const unsigned bi = tile / tpb;
    const Bucket *b = bk + bi;
    const long base = (long)(tile - bi * tpb) * 256 * U;
#pragma unroll
    for (int s = 0; s < R; ++s) {
      const f4 *src = b->src[s] + base;
#pragma unroll
      for (int u = 0; u < U; ++u)
        glds16(src + u * 256 + threadIdx.x, (L4 *)(lds + (s * U + u) * 256 + wave * 64));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    f4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      r[u] = lds[(0 * U + u) * 256 + threadIdx.x];
#pragma unroll
      for (int s = 1; s < R; ++s) r[u] = r[u] + lds[(s * U + u) * 256 + threadIdx.x];
    }
#pragma unroll
    for (int d = 0; d < R; ++d) {
      G4 *dst = (G4 *)b->dst[d] + base;
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_nontemporal_store(r[u], dst + u * 256 + threadIdx.x);
    }
    __syncthreads();  // WAR on the LDS rows before the next pass's DMA
  }
}

// persistent, double-buffered: the DMA of the next tile is issued before the current one is
// waited for; vmcnt counted (R glds per tile per lane; the 8 stores of the previous tile were
// issued before the next DMA, so waiting down to R outstanding retires the current tile)
__global__ __launch_bounds__(256) void fold_glds_pipe(const Bucket *__restrict__ bk, unsigned tpb, unsigned ntiles) {
  __shared__ f4 lds[2][R * 256];
  unsigned tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto issue = [&](unsigned t, int buf) {
    const unsigned bi = t / tpb;
    const long base = (long)(t - bi * tpb) * 256;
    const Bucket *b = bk + bi;
#pragma unroll
    for (int s = 0; s < R; ++s) glds16(b->src[s] + base + threadIdx.x, (L4 *)(lds[buf] + s * 256 + (threadIdx.x & ~63u)));
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
    const unsigned bi = tile / tpb;
    const long base = (long)(tile - bi * tpb) * 256;
    const Bucket *b = bk + bi;
#pragma unroll
    for (int d = 0; d < R; ++d) __builtin_nontemporal_store(r, (G4 *)b->dst[d] + base + threadIdx.x);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's reads of `buf` are done before it is re-filled
  }
}

// copy with the fold's traffic mix (1 byte written per byte read): nt loads to VGPRs / glds
__global__ void copy_nt(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load((const G4 *)a + i), (G4 *)b + i);
}
__global__ __launch_bounds__(256) void copy_glds(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  __shared__ f4 lds[8 * 256];
  const long step = (long)gridDim.x * 256 * 8;
  for (long i0 = (long)blockIdx.x * 256 * 8; i0 < n; i0 += step) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      glds16(a + i0 + k * 256 + threadIdx.x, (L4 *)(lds + k * 256 + (threadIdx.x & ~63u)));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(lds[k * 256 + threadIdx.x], (G4 *)b + i0 + k * 256 + threadIdx.x);
    __syncthreads();
  }
}
// the production fold's body with plain (write-back) stores instead of nt
template <int U>
__global__ __launch_bounds__(256) void fold_plainst(const Bucket *__restrict__ bk, unsigned tpb, unsigned ntiles) {
  for (unsigned tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const unsigned bi = tile / tpb;
    const Bucket *b = bk + bi;
    const long base = (long)(tile - bi * tpb) * 256 * U;
    f4 x[U][R];
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) x[u][s] = __builtin_nontemporal_load((const G4 *)b->src[s] + base + u * 256 + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int s = 1; s < R; ++s) x[u][0] = x[u][0] + x[u][s];
#pragma unroll
    for (int d = 0; d < R; ++d)
#pragma unroll
      for (int u = 0; u < U; ++u) *((G4 *)b->dst[d] + base + u * 256 + threadIdx.x) = x[u][0];
  }
}

__global__ void read_nt(const f4 *__restrict__ a, long n, float *out) {
  f4 acc = {0, 0, 0, 0};
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    acc += __builtin_nontemporal_load((const G4 *)a + i);
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

// each workgroup streams 8 x 4 KiB per pass into LDS, reads one vector back per pass
__global__ __launch_bounds__(256) void read_glds(const f4 *__restrict__ a, long n, float *out) {
  __shared__ f4 lds[8 * 256];
  f4 acc = {0, 0, 0, 0};
  const long step = (long)gridDim.x * 256 * 8;
  for (long i0 = (long)blockIdx.x * 256 * 8; i0 < n; i0 += step) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
      glds16(a + i0 + k * 256 + threadIdx.x, (L4 *)(lds + k * 256 + (threadIdx.x & ~63u)));
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
  long mib = argc > 1 ? atol(argv[1]) : 16;
  int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 20;
  long S = mib << 20, C = S / 16 / R;  // vectors per chunk
  int nsets = std::max<long>(2, (640L << 20) / (2 * R * S) + 1);
  std::vector<Bucket *> dbk(nsets);
  std::vector<emac_bucket *> ebk(nsets);
  for (int st = 0; st < nsets; st++) {
    f4 *send[R], *recv[R];
    for (int r = 0; r < R; r++) {
      CHECK(hipMalloc(&send[r], S));
      CHECK(hipMalloc(&recv[r], S));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, send[r], S / 16, 977u * st + r);
    }
    Bucket hb[R];
    emac_bucket eb[R];
    memset(eb, 0, sizeof(eb));
    for (int c = 0; c < R; c++) {
      for (int t = 0; t < R; t++) hb[c].src[t] = send[(c + t) % R] + c * C;
      for (int d = 0; d < R; d++) hb[c].dst[d] = recv[d] + c * C;
      hb[c].nvec = C;
      for (int t = 0; t < R; t++) eb[c].src[t] = hb[c].src[t];
      for (int d = 0; d < R; d++) eb[c].dst[d] = hb[c].dst[d];
      eb[c].count = C * 4;
      eb[c].nvec = C;
      eb[c].ndst = R;
    }
    CHECK(hipMalloc(&dbk[st], sizeof(hb)));
    CHECK(hipMemcpy(dbk[st], hb, sizeof(hb), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&ebk[st], sizeof(eb)));
    CHECK(hipMemcpy(ebk[st], eb, sizeof(eb), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = R;
  emac_codes tcodes;
  memset(&tcodes, 0, sizeof(tcodes));
  tcodes.nlev = 3;
  tcodes.nleaf = R;
  for (int t = 0; t < R; t++) {
    for (int l = 0; l < 3; l++)
      if (t % (2 << l) == 0) tcodes.first[t] |= (unsigned char)(1 << l);
    tcodes.close[t] = t % 8 == 7 ? 3 : t % 4 == 3 ? 2 : t % 2 == 1 ? 1 : 0;
  }
  f4 *ca;
  long cn = 2 * R * S / 16;  // same bytes as one fold launch moves
  CHECK(hipMalloc(&ca, 2 * cn * 16));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, ca, 2 * cn, 4242u);
  float *dummy;
  CHECK(hipMalloc(&dummy, 64));
  CHECK(hipDeviceSynchronize());
  int k = 0;
  struct V {
    const char *name;
    int kind;
    std::vector<float> us;
  };
  const bool quick = getenv("LDSBENCH_QUICK") != nullptr;
  std::vector<V> vs = {{"u2_vec_burst", 20, {}}, {"u2_src_burst", 21, {}}, {"u2_vec_sleep1", 22, {}},
                       {"u2_src_sleep1", 23, {}}, {"u2_vec_sleep2", 24, {}}, {"u2_src_sleep2", 25, {}},
                       {"u2_vec_sleep3", 26, {}}, {"u2_src_sleep3", 27, {}}, {"u4_src_burst", 31, {}},
                       {"u4_src_sleep1", 33, {}}, {"u4_src_sleep2", 35, {}},
                       {"prod_u2", 0, {}},   {"prod_u4", 1, {}},   {"read_nt", 2, {}},  {"read_glds", 3, {}},
                       {"glds_u1", 4, {}},   {"glds_u2", 5, {}},   {"glds_pipe", 6, {}}, {"glds_pipe_g512", 7, {}},
                       {"copy_nt", 8, {}},   {"copy_glds", 9, {}}, {"fold_plainst_u2", 10, {}}};
  if (getenv("LDSBENCH_TREE"))
    vs = {{"tree_u2_burst", 41, {}}, {"tree_u2_sleep1", 43, {}}, {"tree_u2_sleep2", 45, {}},
          {"tree_u2_sleep3", 47, {}}, {"tree_u4_burst", 51, {}}, {"tree_u4_sleep2", 55, {}},
          {"u4_src_sleep2", 35, {}}, {"u2_src_burst", 21, {}}};
  else if (quick) vs = {{"u2_src_burst", 21, {}}, {"u2_src_sleep1", 23, {}}, {"u2_src_sleep2", 25, {}},
                   {"u2_src_sleep3", 27, {}}, {"u4_src_burst", 31, {}}, {"u4_src_sleep1", 33, {}},
                   {"u4_src_sleep2", 35, {}}, {"u4_src_sleep3", 37, {}}, {"copy_nt", 8, {}}};
  auto run = [&](int kind, int set, int i) {
    switch (kind) {
    case 0:
    case 1: {
      const int U = kind == 0 ? 2 : 4;
      const long tpb = C / (256 * U);
      emac::Launch L = {&codes, ebk[set], R, tpb * R, tpb, 1, nullptr, 0, s};
      if (U == 2)
        emac::launch_one<float, EMAC_SUM, R, 2, false, R>(L);
      else
        emac::launch_one<float, EMAC_SUM, R, 4, false, R>(L);
      break;
    }
    case 20: case 21: case 22: case 23: case 24: case 25: case 26: case 27: {
      // production template, U = 2, load issue schedule ISSUE = kind - 20
      const long tpb = C / 512;
      const dim3 g((unsigned)std::min<long>(tpb * R, 8192));
#define ISS(i) case 20 + i: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, false, R, i>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, codes); break;
      switch (kind) { ISS(0) ISS(1) ISS(2) ISS(3) ISS(4) ISS(5) ISS(6) ISS(7) }
#undef ISS
      break;
    }
    case 41: case 43: case 45: case 47: case 51: case 55: {
      // binary-tree codes (radix chain -2 -2 -2): the production TREE template, U = 2 or 4
      const int U = kind >= 51 ? 4 : 2;
      const long tpb = C / (256 * U);
      const dim3 g((unsigned)std::min<long>(tpb * R, 8192));
      switch (kind) {
      case 41: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, true, R, 1>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, tcodes); break;
      case 43: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, true, R, 3>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, tcodes); break;
      case 45: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, true, R, 5>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, tcodes); break;
      case 47: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, true, R, 7>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, tcodes); break;
      case 51: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, true, R, 1>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, tcodes); break;
      case 55: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, true, R, 5>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, tcodes); break;
      }
      break;
    }
    case 31: case 33: case 35: case 37: {
      const long tpb = C / 1024;
      const dim3 g((unsigned)std::min<long>(tpb * R, 8192));
      if (kind == 31) hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, false, R, 1>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, codes);
      if (kind == 33) hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, false, R, 3>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, codes);
      if (kind == 35) hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, false, R, 5>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, codes);
      if (kind == 37) hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, false, R, 7>), g, dim3(256), 0, s, ebk[set], R, tpb * R, tpb, 1, codes);
      break;
    }
    case 2: hipLaunchKernelGGL(read_nt, dim3(8192), dim3(256), 0, s, ca + (i & 1) * cn, cn, dummy); break;
    case 3: hipLaunchKernelGGL(read_glds, dim3(2048), dim3(256), 0, s, ca + (i & 1) * cn, cn, dummy); break;
    case 4: {
      unsigned tpb = C / 256;
      hipLaunchKernelGGL(fold_glds<1>, dim3(std::min<unsigned>(tpb * R, 8192)), dim3(256), 0, s, dbk[set], tpb, tpb * R);
      break;
    }
    case 5: {
      unsigned tpb = C / 512;
      hipLaunchKernelGGL(fold_glds<2>, dim3(std::min<unsigned>(tpb * R, 8192)), dim3(256), 0, s, dbk[set], tpb, tpb * R);
      break;
    }
    case 6:
    case 7: {
      unsigned tpb = C / 256;
      hipLaunchKernelGGL(fold_glds_pipe, dim3(kind == 6 ? 1024 : 512), dim3(256), 0, s, dbk[set], tpb, tpb * R);
      break;
    }
    case 8: hipLaunchKernelGGL(copy_nt, dim3(8192), dim3(256), 0, s, ca + (i & 1) * cn, ca + ((i & 1) ^ 1) * cn + cn / 2, cn / 2); break;
    case 9: hipLaunchKernelGGL(copy_glds, dim3(2048), dim3(256), 0, s, ca + (i & 1) * cn, ca + ((i & 1) ^ 1) * cn + cn / 2, cn / 2); break;
    case 10: {
      unsigned tpb = C / 512;
      hipLaunchKernelGGL(fold_plainst<2>, dim3(std::min<unsigned>(tpb * R, 8192)), dim3(256), 0, s, dbk[set], tpb, tpb * R);
      break;
    }
    }
  };
  // correctness: every fold variant must produce prod_u2's bytes for one chunk
  {
    std::vector<char> ref(C * 16), got(C * 16);
    Bucket hb;
    CHECK(hipMemcpy(&hb, dbk[0] + 3, sizeof(hb), hipMemcpyDeviceToHost));
    for (int kind : {0, 1, 4, 5, 6, 7, 10, 20, 21, 22, 23, 24, 25, 26, 27, 31, 33, 35, 37}) {
      CHECK(hipMemset(hb.dst[5], 0, C * 16));
      run(kind, 0, 0);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(kind ? got.data() : ref.data(), hb.dst[5], C * 16, hipMemcpyDeviceToHost));
      if (kind && memcmp(ref.data(), got.data(), C * 16)) printf("MISMATCH kind %d\n", kind);
    }
  }
  {
    std::vector<char> ref(C * 16), got(C * 16);
    Bucket hb;
    CHECK(hipMemcpy(&hb, dbk[0] + 3, sizeof(hb), hipMemcpyDeviceToHost));
    for (int kind : {41, 43, 45, 47, 51, 55}) {
      CHECK(hipMemset(hb.dst[5], 0, C * 16));
      run(kind, 0, 0);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(kind == 41 ? ref.data() : got.data(), hb.dst[5], C * 16, hipMemcpyDeviceToHost));
      if (kind != 41 && memcmp(ref.data(), got.data(), C * 16)) printf("MISMATCH tree kind %d\n", kind);
    }
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; rd++)
    for (auto &v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) run(v.kind, (k++) % nsets, i);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000 / per);
    }
  CHECK(hipGetLastError());
  auto med = [](std::vector<float> x) {
    std::sort(x.begin(), x.end());
    return x[x.size() / 2];
  };
  double bytes = 2.0 * R * S;
  printf("# %ld MiB per rank, R=%d, %d sets, %d rounds x %d launches; GB/s = 2*R*S / t\n", mib, R, nsets, rounds, per);
  for (auto &v : vs)
    printf("%-16s median %8.2f us  min %8.2f us  %7.1f GB/s (best %7.1f)\n", v.name, med(v.us),
           *std::min_element(v.us.begin(), v.us.end()), bytes / med(v.us) / 1e3,
           bytes / *std::min_element(v.us.begin(), v.us.end()) / 1e3);
  return 0;
}
