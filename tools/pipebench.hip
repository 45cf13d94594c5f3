// pipebench.hip -- round-3 A/B harness: can a persistent, register-pipelined fold (the loads of
// tile t+1 issued before tile t is folded and stored) beat the production grid-stride fold on the
// local fold (8 x C -> 1) and the node fold (8 x C -> 8 x C), and which copy kernel is the real
// 1:1 read/write ceiling? One process, interleaved rounds, median per variant.
//   prod_local / prod_node   fold_kernel<float, SUM, 8, U=4, linear, D, burst> as the library runs it
//   pipe_local_uU_kK         persistent (K workgroups per CU), contiguous tile ranges, U vectors per
//                            lane per leaf, double-buffered in registers
//   pipe_node_uU_kK          the same with the 8-way fan-out store
//   copy_*                   1:1 copies over 9 x C bytes read + written (ceiling candidates)
//   read_glds                read-only LDS-DMA stream (the read ceiling of bench.py)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/pipebench.hip -o tools/pipebench
// Run:   tools/pipebench [chunk MiB = 32] [rounds = 7] [launches per round = 10]
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
typedef __attribute__((address_space(3))) f4 L4;
constexpr int R = 8;

struct Job {
  const f4 *src[R];
  f4 *dst[R];
  long nvec;  // vectors per leaf
};

// Persistent pipelined fold: workgroup w owns tiles [w * T / G, (w + 1) * T / G) (contiguous,
// so consecutive passes of one workgroup stream consecutive addresses); registers a / b hold
// the current and the next tile's leaves.
template <int U, int D>
__global__ __launch_bounds__(256) void pipe_fold(Job j, long ntiles) {
  const long t0 = (long)blockIdx.x * ntiles / gridDim.x, t1 = (long)(blockIdx.x + 1) * ntiles / gridDim.x;
  if (t0 >= t1) return;
  const G4 *src[R];
#pragma unroll
  for (int s = 0; s < R; ++s) src[s] = (const G4 *)j.src[s];
  f4 a[U][R], b[U][R];
  auto load = [&](f4 (&x)[U][R], long t) {
    const long base = t * 256 * U + threadIdx.x;
#pragma unroll
    for (int s = 0; s < R; ++s)
#pragma unroll
      for (int u = 0; u < U; ++u) x[u][s] = __builtin_nontemporal_load(src[s] + base + u * 256);
  };
  auto fold_store = [&](f4 (&x)[U][R], long t) {
    const long base = t * 256 * U + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f4 r = x[u][0];
#pragma unroll
      for (int s = 1; s < R; ++s) r = r + x[u][s];
#pragma unroll
      for (int d = 0; d < D; ++d) __builtin_nontemporal_store(r, (G4 *)j.dst[d] + base + u * 256);
    }
  };
  load(a, t0);
  long t = t0;
  for (; t + 1 < t1; t += 2) {
    load(b, t + 1);
    fold_store(a, t);
    if (t + 2 < t1) load(a, t + 2);
    fold_store(b, t + 1);
  }
  if (t < t1) fold_store(a, t);
}

__device__ __forceinline__ void glds16(const f4 *g, L4 *l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                   (__attribute__((address_space(3))) void *)l, 16, 0, 2 /* nt */);
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

// copies: K vectors per lane in flight per pass, grid-stride (NT: nontemporal loads / stores)
template <int K, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void copy_k(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  const long step = (long)gridDim.x * 256 * K;
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
    f4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = NTL ? __builtin_nontemporal_load((const G4 *)a + i0 + k * 256) : ((const G4 *)a)[i0 + k * 256];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (NTS)
        __builtin_nontemporal_store(v[k], (G4 *)b + i0 + k * 256);
      else
        ((G4 *)b)[i0 + k * 256] = v[k];
    }
  }
}

// persistent pipelined copy (contiguous ranges, double-buffered in registers)
template <int K>
__global__ __launch_bounds__(256) void copy_pipe(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  const long T = n / (256 * K);
  const long t0 = (long)blockIdx.x * T / gridDim.x, t1 = (long)(blockIdx.x + 1) * T / gridDim.x;
  f4 x[K], y[K];
  auto ld = [&](f4 (&v)[K], long t) {
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load((const G4 *)a + t * 256 * K + k * 256 + threadIdx.x);
  };
  auto st = [&](f4 (&v)[K], long t) {
#pragma unroll
    for (int k = 0; k < K; ++k) __builtin_nontemporal_store(v[k], (G4 *)b + t * 256 * K + k * 256 + threadIdx.x);
  };
  if (t0 >= t1) return;
  ld(x, t0);
  long t = t0;
  for (; t + 1 < t1; t += 2) {
    ld(y, t + 1);
    st(x, t);
    if (t + 2 < t1) ld(x, t + 2);
    st(y, t + 1);
  }
  if (t < t1) st(x, t);
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
  const int nsets = std::max<long>(2, (768L << 20) / (2 * R * (mib << 20)) + 1);
  std::vector<Job> jobs(nsets);
  std::vector<emac_bucket *> eloc(nsets), enode(nsets);
  for (int st = 0; st < nsets; st++) {
    emac_bucket eb, en;
    memset(&eb, 0, sizeof(eb));
    memset(&en, 0, sizeof(en));
    for (int s = 0; s < R; s++) {
      f4 *p, *q;
      CHECK(hipMalloc(&p, C * 16));
      CHECK(hipMalloc(&q, C * 16));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, p, C, 977u * st + s);
      jobs[st].src[s] = p;
      jobs[st].dst[s] = q;
      eb.src[s] = en.src[s] = p;
      en.dst[s] = q;
    }
    jobs[st].nvec = C;
    eb.dst[0] = jobs[st].dst[0];
    eb.ndst = 1;
    en.ndst = R;
    eb.count = en.count = C * 4;
    eb.nvec = en.nvec = C;
    CHECK(hipMalloc(&eloc[st], sizeof(eb)));
    CHECK(hipMemcpy(eloc[st], &eb, sizeof(eb), hipMemcpyHostToDevice));
    CHECK(hipMalloc(&enode[st], sizeof(en)));
    CHECK(hipMemcpy(enode[st], &en, sizeof(en), hipMemcpyHostToDevice));
  }
  f4 *ca;
  const long cn = (long)(R + 1) * C;  // the local fold's bytes: copies move cn read + cn written
  CHECK(hipMalloc(&ca, 4 * cn * 16));
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, ca, 4 * cn, 4242u);
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
    std::string name;
    int kind, u, k;
    double bytes;
    std::vector<float> us;
  };
  const double lb = (double)(R + 1) * C * 16, nb = (double)2 * R * C * 16, cb = 2.0 * cn * 16;
  std::vector<V> vs = {{"prod_local_u4", 0, 4, 0, lb, {}}, {"prod_node_u4", 1, 4, 0, nb, {}}, {"prod_node_u2", 1, 2, 0, nb, {}}};
  for (int u : {1, 2})
    for (int k : {1, 2, 3, 4}) {
      vs.push_back({"pipe_local_u" + std::to_string(u) + "_k" + std::to_string(k), 2, u, k, lb, {}});
      vs.push_back({"pipe_node_u" + std::to_string(u) + "_k" + std::to_string(k), 3, u, k, nb, {}});
    }
  vs.push_back({"copy_k1_nt_nt", 10, 1, 0, cb, {}});
  vs.push_back({"copy_k4_nt_nt", 11, 4, 0, cb, {}});
  vs.push_back({"copy_k4_pl_pl", 12, 4, 0, cb, {}});
  vs.push_back({"copy_k4_nt_pl", 13, 4, 0, cb, {}});
  vs.push_back({"copy_k8_nt_nt", 14, 8, 0, cb, {}});
  vs.push_back({"copy_pipe_k4_g512", 15, 4, 2, cb, {}});
  vs.push_back({"copy_pipe_k4_g1024", 15, 4, 4, cb, {}});
  vs.push_back({"copy_pipe_k2_g1024", 16, 2, 4, cb, {}});
  vs.push_back({"read_glds", 20, 0, 0, (double)2 * cn * 16, {}});
  auto run = [&](const V &v, int set, int i) {
    switch (v.kind) {
    case 0: {
      const long nt = C / (256L * 4);
      hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, 0, 1, 1>), dim3((unsigned)std::min<long>(nt, 8192)), dim3(256), 0, s,
                         eloc[set], 1, nt, nt, 1, codes, (const unsigned *)nullptr, R);
      break;
    }
    case 1: {
      const long nt = C / (256L * v.u);
      if (v.u == 4)
        hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 4, 0, R, 1>), dim3((unsigned)std::min<long>(nt, 8192)), dim3(256), 0, s,
                           enode[set], 1, nt, nt, 1, codes, (const unsigned *)nullptr, R);
      else
        hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, 2, 0, R, 1>), dim3((unsigned)std::min<long>(nt, 8192)), dim3(256), 0, s,
                           enode[set], 1, nt, nt, 1, codes, (const unsigned *)nullptr, R);
      break;
    }
    case 2:
    case 3: {
      const long nt = C / (256L * v.u);
      const dim3 g(256 * v.k);
      if (v.kind == 2) {
        if (v.u == 1) hipLaunchKernelGGL((pipe_fold<1, 1>), g, dim3(256), 0, s, jobs[set], nt);
        else hipLaunchKernelGGL((pipe_fold<2, 1>), g, dim3(256), 0, s, jobs[set], nt);
      } else {
        if (v.u == 1) hipLaunchKernelGGL((pipe_fold<1, R>), g, dim3(256), 0, s, jobs[set], nt);
        else hipLaunchKernelGGL((pipe_fold<2, R>), g, dim3(256), 0, s, jobs[set], nt);
      }
      break;
    }
    case 10: hipLaunchKernelGGL((copy_k<1, true, true>), dim3(8192), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 11: hipLaunchKernelGGL((copy_k<4, true, true>), dim3(4096), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 12: hipLaunchKernelGGL((copy_k<4, false, false>), dim3(4096), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 13: hipLaunchKernelGGL((copy_k<4, true, false>), dim3(4096), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 14: hipLaunchKernelGGL((copy_k<8, true, true>), dim3(2048), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 15: hipLaunchKernelGGL((copy_pipe<4>), dim3(256 * v.k), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 16: hipLaunchKernelGGL((copy_pipe<2>), dim3(256 * v.k), dim3(256), 0, s, ca + (i & 1) * 2 * cn, ca + (i & 1) * 2 * cn + cn, cn); break;
    case 20: hipLaunchKernelGGL(read_glds, dim3(2048), dim3(256), 0, s, ca + (i & 1) * 2 * cn, 2 * cn, dummy); break;
    }
  };
  // correctness of the pipelined kernels against the production local / node fold (bitwise)
  {
    std::vector<float> want((size_t)C * 4), got((size_t)C * 4);
    run(vs[0], 0, 0);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(want.data(), jobs[0].dst[0], C * 16, hipMemcpyDeviceToHost));
    for (const V &v : vs) {
      if (v.kind != 2 && v.kind != 3) continue;
      CHECK(hipMemset(jobs[0].dst[0], 0, C * 16));
      CHECK(hipMemset(jobs[0].dst[R - 1], 0, C * 16));
      run(v, 0, 0);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(got.data(), jobs[0].dst[v.kind == 3 ? R - 1 : 0], C * 16, hipMemcpyDeviceToHost));
      if (memcmp(got.data(), want.data(), C * 16)) printf("MISMATCH %s\n", v.name.c_str());
    }
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; w++)
    for (const V &v : vs) run(v, w % nsets, w);
  CHECK(hipStreamSynchronize(s));
  for (int r = 0; r < rounds; r++)
    for (V &v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) run(v, i % nsets, i);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / per);
    }
  printf("chunk %ld MiB per leaf, %d sets, %d rounds x %d launches (median, min, max us; TB/s of algorithmic bytes)\n", mib,
         nsets, rounds, per);
  for (V &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-22s %9.2f %9.2f %9.2f  %6.3f TB/s  %.3f of 8\n", v.name.c_str(), med, v.us.front(), v.us.back(),
           v.bytes / med / 1e6, v.bytes / med / 1e6 / 8.0);
  }
  return 0;
}
