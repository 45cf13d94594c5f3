// occbench.hip -- occupancy and grid shape of the node-form fold (R = 8 leaves, fan-out 8, float
// SUM, U = 4, staggered issue): the production kernel holds 140 VGPRs, i.e. 3 waves per SIMD, so
// the 1024 tiles of a 16 MiB-per-rank launch do not fit the chip at once (768 resident). Variants:
//   prod          emac::fold_kernel<float, SUM, 8, 4, false, 8, 5>, grid = tiles (production)
//   occ4          the same body with amdgpu_waves_per_eu(4): <= 128 VGPRs, every tile resident
//   occ4_burst    occ4 with every load back to back
//   grid768       production kernel, grid = 768 (one resident round, grid-stride over the rest)
//   grid512       production kernel, grid = 512
// One process, interleaved rounds; every variant's bytes checked against prod's.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/occbench.hip -o tools/occbench
// Run:   tools/occbench [MiB per rank = 16] [rounds = 7] [launches per round = 20]
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

constexpr int R = 8, U = 4;

template <int ISSUE>
__global__ __launch_bounds__(EMAC_BLOCK) __attribute__((amdgpu_waves_per_eu(4))) void fold_occ4(
    const emac_bucket *__restrict__ bk, long ntiles, long tpb, emac_codes codes) {
  constexpr long TILE = (long)EMAC_BLOCK * U;
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bi = (int)((unsigned)tile / (unsigned)tpb);
    const long t = tile - (long)bi * tpb;
    emac::fold_vectors<float, EMAC_SUM, R, U, false, R, true, ISSUE>(bk + bi, t * TILE, 0, codes);
  }
}

__global__ void fill_random(float *p, long n, unsigned seed) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed * 2246822519u;
    x ^= x >> 13;
    x *= 3266489917u;
    x ^= x >> 16;
    p[i] = (float)(x & 0xFFFFFF) / 8388608.0f - 1.0f;
  }
}

int main(int argc, char **argv) {
  long mib = argc > 1 ? atol(argv[1]) : 16;
  int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 20;
  long S = mib << 20, C = S / 16 / R;  // vectors per chunk
  int nsets = std::max<long>(2, (640L << 20) / (2 * R * S) + 1);
  std::vector<emac_bucket *> ebk(nsets);
  std::vector<float *> recv0(nsets);
  for (int st = 0; st < nsets; st++) {
    float *send[R], *recv[R];
    for (int r = 0; r < R; r++) {
      CHECK(hipMalloc(&send[r], S));
      CHECK(hipMalloc(&recv[r], S));
      hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, send[r], S / 4, 977u * st + r);
    }
    recv0[st] = recv[5];
    emac_bucket eb[R];
    memset(eb, 0, sizeof(eb));
    for (int c = 0; c < R; c++) {
      for (int t = 0; t < R; t++) eb[c].src[t] = send[(c + t) % R] + c * C * 4;
      for (int d = 0; d < R; d++) eb[c].dst[d] = recv[d] + c * C * 4;
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
  const long tpb = C / (EMAC_BLOCK * U), ntiles = tpb * R;
  struct V {
    const char *name;
    int kind;
    std::vector<float> us;
  };
  std::vector<V> vs = {{"prod", 0, {}}, {"occ4", 1, {}}, {"occ4_burst", 2, {}}, {"grid768", 3, {}}, {"grid512", 4, {}}};
  auto run = [&](int kind, int set) {
    const unsigned g = (unsigned)std::min<long>(ntiles, 8192);
    switch (kind) {
    case 0: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, false, R, 5>), dim3(g), dim3(EMAC_BLOCK), 0, s, ebk[set], R, ntiles, tpb, 1, codes); break;
    case 1: hipLaunchKernelGGL(fold_occ4<5>, dim3(g), dim3(EMAC_BLOCK), 0, s, ebk[set], ntiles, tpb, codes); break;
    case 2: hipLaunchKernelGGL(fold_occ4<1>, dim3(g), dim3(EMAC_BLOCK), 0, s, ebk[set], ntiles, tpb, codes); break;
    case 3: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, false, R, 5>), dim3(std::min<long>(ntiles, 768)), dim3(EMAC_BLOCK), 0, s, ebk[set], R, ntiles, tpb, 1, codes); break;
    case 4: hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, U, false, R, 5>), dim3(std::min<long>(ntiles, 512)), dim3(EMAC_BLOCK), 0, s, ebk[set], R, ntiles, tpb, 1, codes); break;
    }
  };
  {
    std::vector<char> ref(S), got(S);
    for (auto &v : vs) {
      CHECK(hipMemset(recv0[0], 0, S));
      run(v.kind, 0);
      CHECK(hipStreamSynchronize(s));
      CHECK(hipMemcpy(v.kind ? got.data() : ref.data(), recv0[0], S, hipMemcpyDeviceToHost));
      if (v.kind && memcmp(ref.data(), got.data(), S)) printf("MISMATCH %s\n", v.name);
    }
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int k = 0;
  for (int rd = 0; rd < rounds; rd++)
    for (auto &v : vs) {
      CHECK(hipEventRecord(e0, s));
      for (int i = 0; i < per; i++) run(v.kind, (k++) % nsets);
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
  printf("# %ld MiB per rank, R=%d, %ld tiles, %d sets, %d rounds x %d launches; GB/s = 2*R*S / t\n", mib, R, ntiles,
         nsets, rounds, per);
  for (auto &v : vs)
    printf("%-12s median %8.2f us  min %8.2f us  %7.1f GB/s (best %7.1f)\n", v.name, med(v.us),
           *std::min_element(v.us.begin(), v.us.end()), bytes / med(v.us) / 1e3,
           bytes / *std::min_element(v.us.begin(), v.us.end()) / 1e3);
  return 0;
}
