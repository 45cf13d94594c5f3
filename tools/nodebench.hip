// nodebench.hip -- launch-schedule A/B of the NODE-form fold (R = 8 ranks in one HBM: 8 owner
// chunks, each 8 leaves -> 8 destinations), the production fold_kernel template, interleaved
// rounds in one process, median per variant. Run on several leases (fresh boxes) to separate a
// schedule's win from the box-to-box spread (emac_gpu_pick_unroll, fold.hip).
//   uU_iI   fold_kernel<float, SUM, 8, U, linear, fan-out 8, ISSUE I>  (I = 1 burst, 5 / 3 s_sleep
//           2 / 1 after every 4 loads)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/nodebench.hip -o tools/nodebench
// Run:   tools/nodebench [MiB per rank = 16] [rounds = 9] [launches per round = 10]
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
constexpr int R = 8;

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
  const long mib = argc > 1 ? atol(argv[1]) : 16;
  const int rounds = argc > 2 ? atoi(argv[2]) : 9, per = argc > 3 ? atoi(argv[3]) : 10;
  const long S = mib << 20, C = S / 16 / R;  // vectors per owner chunk
  const int nsets = std::max<long>(2, (768L << 20) / (2 * R * S) + 1);
  std::vector<emac_bucket *> ebk(nsets);
  for (int st = 0; st < nsets; st++) {
    f4 *send[R], *recv[R];
    for (int r = 0; r < R; r++) {
      CHECK(hipMalloc(&send[r], S));
      CHECK(hipMalloc(&recv[r], S));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, send[r], S / 16, 977u * st + r);
    }
    emac_bucket eb[R];
    memset(eb, 0, sizeof(eb));
    for (int c = 0; c < R; c++) {
      for (int t = 0; t < R; t++) eb[c].src[t] = send[(c + t) % R] + c * C;
      for (int d = 0; d < R; d++) eb[c].dst[d] = recv[d] + c * C;
      eb[c].count = C * 4;
      eb[c].nvec = C;
      eb[c].ndst = R;
    }
    CHECK(hipMalloc(&ebk[st], sizeof(eb)));
    CHECK(hipMemcpy(ebk[st], eb, sizeof(eb), hipMemcpyHostToDevice));
  }
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = R;
  CHECK(hipDeviceSynchronize());
  struct V {
    const char *name;
    int u, issue;
    std::vector<float> us;
  };
  std::vector<V> vs = {{"u2_i1", 2, 1, {}}, {"u4_i1", 4, 1, {}}, {"u4_i5", 4, 5, {}}, {"u2_i5", 2, 5, {}},
                       {"u4_i3", 4, 3, {}}, {"u1_i1", 1, 1, {}}};
  auto run = [&](const V &v, int set) {
    const long tpb = C / (256L * v.u);
    const dim3 g((unsigned)std::min<long>(tpb * R, 8192));
#define NB_K(uu, ii)                                                                                             \
  if (v.u == uu && v.issue == ii) {                                                                              \
    hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, uu, 0, R, ii>), g, dim3(256), 0, s, ebk[set], R,    \
                       tpb * R, tpb, 1, codes, (const unsigned *)nullptr, R);                                    \
  }
    NB_K(2, 1) NB_K(4, 1) NB_K(4, 5) NB_K(2, 5) NB_K(4, 3) NB_K(1, 1)
#undef NB_K
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int k = 0;
  for (auto &v : vs)
    for (int i = 0; i < 3; i++) run(v, (k++) % nsets);
  CHECK(hipStreamSynchronize(s));
  for (int rd = 0; rd < rounds; rd++)
    for (auto &v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) run(v, (k++) % nsets);
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1000.f / per);
    }
  CHECK(hipGetLastError());
  const double bytes = 2.0 * R * S;
  printf("node fold: %d ranks x %ld MiB, %d sets, %d rounds x %d launches (median us, GB/s of %.0f MB)\n", R, mib, nsets,
         rounds, per, bytes / 1e6);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-8s %9.2f us  %7.1f GB/s  (min %.2f max %.2f)\n", v.name, med, bytes / (med * 1e-6) / 1e9, v.us.front(),
           v.us.back());
  }
  return 0;
}
