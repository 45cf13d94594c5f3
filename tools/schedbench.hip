// schedbench.hip -- round-3 A/B harness for the fold's cache policy and unroll: the production
// fold_kernel (fold_kernel.hpp) on the node form's real layout (R = 8 ranks' send / receive
// buffers of S = 8 C bytes, 8 buckets, every bucket's result fanned out to every rank) and on the
// local fold (8 leaves of C bytes -> 1), with nontemporal or default-policy (allocating) loads /
// stores (ISSUE bits kPlainStore, kPlainLoad), plus the copy and read ceilings of bench.py.
// One process, interleaved rounds, median per variant; buffer sets rotated beyond the 256 MiB
// Infinity Cache.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/schedbench.hip -o tools/schedbench
// Run:   tools/schedbench [chunk KiB = 2048] [rounds = 7] [launches per round = 10]
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
using emac::kPlainLoad;
using emac::kPlainStore;

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

template <int K, bool NT>
__global__ __launch_bounds__(256) void copy_k(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  const long step = (long)gridDim.x * 256 * K;
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
    f4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = NT ? __builtin_nontemporal_load((const G4 *)a + i0 + k * 256) : ((const G4 *)a)[i0 + k * 256];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (NT)
        __builtin_nontemporal_store(v[k], (G4 *)b + i0 + k * 256);
      else
        ((G4 *)b)[i0 + k * 256] = v[k];
    }
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

template <int U, int D, int ISSUE>
void fold(const emac_bucket *b, int nb, long ntiles, long tpb, const emac_codes &c, hipStream_t s) {
  hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, 0, D, ISSUE>), dim3((unsigned)std::min<long>(ntiles, 8192)),
                     dim3(256), 0, s, b, nb, ntiles, tpb, 1, c, (const unsigned *)nullptr, R);
}

int main(int argc, char **argv) {
  const long kib = argc > 1 ? atol(argv[1]) : 2048;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 10;
  const long C = (kib << 10) / 16;  // vectors per chunk (bucket)
  const long S = R * C;             // vectors per rank's message
  const long set_bytes = 2L * R * S * 16;
  const int nsets = (int)std::max<long>(2, (1024L << 20) / set_bytes + 1);
  std::vector<emac_bucket *> dnode(nsets), dloc(nsets);
  std::vector<f4 *> sends(nsets * R), recvs(nsets * R);
  for (int st = 0; st < nsets; st++) {
    std::vector<emac_bucket> bk(R);
    for (int r = 0; r < R; r++) {
      CHECK(hipMalloc(&sends[st * R + r], S * 16));
      CHECK(hipMalloc(&recvs[st * R + r], S * 16));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, sends[st * R + r], S, 977u * st + r);
    }
    for (int c = 0; c < R; c++) {
      memset(&bk[c], 0, sizeof(emac_bucket));
      for (int t = 0; t < R; t++) bk[c].src[t] = sends[st * R + (c + t) % R] + c * C;
      for (int r = 0; r < R; r++) bk[c].dst[r] = recvs[st * R + r] + c * C;
      bk[c].ndst = R;
      bk[c].count = C * 4;
      bk[c].nvec = C;
    }
    CHECK(hipMalloc(&dnode[st], sizeof(emac_bucket) * R));
    CHECK(hipMemcpy(dnode[st], bk.data(), sizeof(emac_bucket) * R, hipMemcpyHostToDevice));
    emac_bucket lb = bk[0];  // the local fold: bucket 0's leaves -> rank 0's receive buffer
    lb.ndst = 1;
    CHECK(hipMalloc(&dloc[st], sizeof(emac_bucket)));
    CHECK(hipMemcpy(dloc[st], &lb, sizeof(emac_bucket), hipMemcpyHostToDevice));
  }
  const long cn = 2L * R * C;  // copy: the node launch's bytes (R C read per bucket x R... = 8 S read, 8 S written)
  const long copy_n = (long)R * S;
  f4 *ca;
  CHECK(hipMalloc(&ca, 2 * 2 * copy_n * 16 > (2L << 30) ? 2 * copy_n * 16 : 4 * copy_n * 16));
  const int csets = 2 * 2 * copy_n * 16 > (2L << 30) ? 1 : 2;
  hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, ca, csets * 2 * copy_n, 4242u);
  (void)cn;
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
    int id;
    double bytes;
    std::vector<float> us;
  };
  const double node_b = 2.0 * R * S * 16, loc_b = (double)(R + 1) * C * 16, copy_b = 2.0 * copy_n * 16;
  std::vector<V> vs = {
      {"node_u4_nt", 0, node_b, {}},        {"node_u4_ps", 1, node_b, {}},   {"node_u4_pls", 2, node_b, {}},
      {"node_u2_nt", 3, node_b, {}},        {"node_u2_ps", 4, node_b, {}},   {"node_u2_pls", 5, node_b, {}},
      {"node_u4_nt_stagger", 6, node_b, {}}, {"node_u4_ps_stagger", 7, node_b, {}},
      {"local_u4_nt", 10, loc_b, {}},       {"local_u4_ps", 11, loc_b, {}},  {"local_u4_pls", 12, loc_b, {}},
      {"local_u2_nt", 13, loc_b, {}},       {"local_u2_ps", 14, loc_b, {}},  {"local_u8_nt", 15, loc_b, {}},
      {"copy_k4_nt", 20, copy_b, {}},       {"copy_k4_plain", 21, copy_b, {}}, {"copy_k8_nt", 22, copy_b, {}},
      {"read_glds", 30, copy_b, {}}};
  auto run = [&](const V &v, int i) {
    const int st = i % nsets;
    const long t4 = C / (256L * 4), t2 = C / (256L * 2), t8 = C / (256L * 8);
    f4 *ca0 = ca + (csets > 1 ? (i & 1) * 2 * copy_n : 0);
    switch (v.id) {
    case 0: fold<4, R, 1>(dnode[st], R, R * t4, t4, codes, s); break;
    case 1: fold<4, R, 1 | kPlainStore>(dnode[st], R, R * t4, t4, codes, s); break;
    case 2: fold<4, R, 1 | kPlainStore | kPlainLoad>(dnode[st], R, R * t4, t4, codes, s); break;
    case 3: fold<2, R, 1>(dnode[st], R, R * t2, t2, codes, s); break;
    case 4: fold<2, R, 1 | kPlainStore>(dnode[st], R, R * t2, t2, codes, s); break;
    case 5: fold<2, R, 1 | kPlainStore | kPlainLoad>(dnode[st], R, R * t2, t2, codes, s); break;
    case 6: fold<4, R, 5>(dnode[st], R, R * t4, t4, codes, s); break;
    case 7: fold<4, R, 5 | kPlainStore>(dnode[st], R, R * t4, t4, codes, s); break;
    case 10: fold<4, 1, 1>(dloc[st], 1, t4, t4, codes, s); break;
    case 11: fold<4, 1, 1 | kPlainStore>(dloc[st], 1, t4, t4, codes, s); break;
    case 12: fold<4, 1, 1 | kPlainStore | kPlainLoad>(dloc[st], 1, t4, t4, codes, s); break;
    case 13: fold<2, 1, 1>(dloc[st], 1, t2, t2, codes, s); break;
    case 14: fold<2, 1, 1 | kPlainStore>(dloc[st], 1, t2, t2, codes, s); break;
    case 15: fold<8, 1, 1>(dloc[st], 1, t8, t8, codes, s); break;
    case 20: hipLaunchKernelGGL((copy_k<4, true>), dim3(4096), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 21: hipLaunchKernelGGL((copy_k<4, false>), dim3(4096), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 22: hipLaunchKernelGGL((copy_k<8, true>), dim3(2048), dim3(256), 0, s, ca0, ca0 + copy_n, copy_n); break;
    case 30: hipLaunchKernelGGL(read_glds, dim3(2048), dim3(256), 0, s, ca0, 2 * copy_n, dummy); break;
    }
  };
  {  // every node variant stores the same bits into every receive buffer
    std::vector<float> want((size_t)S * 4), got((size_t)S * 4);
    run(vs[0], 0);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(want.data(), recvs[R - 1], S * 16, hipMemcpyDeviceToHost));
    for (const V &v : vs) {
      if (v.id >= 10) continue;
      CHECK(hipMemset(recvs[R - 1], 0, S * 16));
      run(v, 0);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(got.data(), recvs[R - 1], S * 16, hipMemcpyDeviceToHost));
      if (memcmp(got.data(), want.data(), S * 16)) printf("MISMATCH %s\n", v.name.c_str());
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
  printf("chunk %ld KiB (%ld KiB per rank, node launch %.1f MiB), %d sets, %d rounds x %d launches: median min max us, TB/s\n",
         kib, kib * R, node_b / 1048576.0, nsets, rounds, per);
  for (V &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-20s %9.2f %9.2f %9.2f  %6.3f TB/s  %.3f of 8\n", v.name.c_str(), med, v.us.front(), v.us.back(),
           v.bytes / med / 1e6, v.bytes / med / 1e6 / 8.0);
  }
  return 0;
}
