// nodeorder.hip -- why does the NODE-form fold (R = 8 ranks in one HBM) lose rate as the message
// grows (16 -> 256 -> 512 MiB per rank)? Interleaved A/B of the production fold_kernel (U 4,
// s_sleep schedule, linear, fan-out 8) over the same buffers with different tile orders, and over
// buffers whose bases are staggered (a diagnostic of address aliasing between the 16 streams):
//   seq_uU_iI  8 buckets (one per owner chunk), tiles of bucket 0 first -- the production layout;
//              U vectors per lane and leaf, ISSUE 1 = burst, 5 = s_sleep 2 after every 4 loads
//   ilK        every owner chunk cut into K-KiB parts, parts of the 8 chunks interleaved (part p of
//              chunk c is bucket p * 8 + c): the resident workgroups spread over all 8 chunks
//   stag       seq, on a second buffer set whose rank r bases are offset by r * (64 KiB + 4 KiB)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/nodeorder.hip -o tools/nodeorder
// Run:   tools/nodeorder [MiB per rank = 256] [rounds = 7] [launches per round = 4]
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
constexpr int R = 8;
constexpr long STAG = 68L << 10;

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

struct Set {
  f4 *send[R], *recv[R];
};

static Set make_set(long S, long stagger, unsigned seed) {
  Set st;
  for (int r = 0; r < R; r++) {
    char *a, *b;
    CHECK(hipMalloc(&a, S + R * stagger));
    CHECK(hipMalloc(&b, S + R * stagger));
    st.send[r] = (f4 *)(a + r * stagger);
    st.recv[r] = (f4 *)(b + r * stagger);
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, st.send[r], S / 16, seed + r);
  }
  return st;
}

// the owner chunks of a set cut into parts of `part` vectors (0: whole chunks), interleaved
static emac_bucket *make_buckets(const Set &st, long C, long part, int U, int *nb) {
  const long TILE = 256L * U;  // vectors per tile
  const long np = part ? C / part : 1, pl = part ? part : C;
  std::vector<emac_bucket> eb((size_t)(np * R));
  memset(eb.data(), 0, eb.size() * sizeof(emac_bucket));
  for (long p = 0; p < np; p++)
    for (int c = 0; c < R; c++) {
      emac_bucket &b = eb[(size_t)(p * R + c)];
      for (int t = 0; t < R; t++) b.src[t] = st.send[(c + t) % R] + c * C + p * pl;
      for (int d = 0; d < R; d++) b.dst[d] = st.recv[d] + c * C + p * pl;
      b.count = pl * 4;
      b.nvec = pl;
      b.ndst = R;
      b.tile0 = (p * R + c) * (pl / TILE);
    }
  emac_bucket *d;
  CHECK(hipMalloc(&d, eb.size() * sizeof(emac_bucket)));
  CHECK(hipMemcpy(d, eb.data(), eb.size() * sizeof(emac_bucket), hipMemcpyHostToDevice));
  *nb = (int)eb.size();
  return d;
}

int main(int argc, char **argv) {
  const long mib = argc > 1 ? atol(argv[1]) : 256;
  const int rounds = argc > 2 ? atoi(argv[2]) : 7, per = argc > 3 ? atoi(argv[3]) : 4;
  const long S = mib << 20, C = S / 16 / R;  // vectors per owner chunk
  const int nsets = (int)std::max<long>(2, (768L << 20) / (2 * R * S) + 1);
  std::vector<Set> plain, stag;
  for (int i = 0; i < nsets; i++) plain.push_back(make_set(S, 0, 977u * i));
  for (int i = 0; i < nsets; i++) stag.push_back(make_set(S, STAG, 977u * i + 500));
  struct V {
    std::string name;
    long part;  // vectors per part (0: whole chunk)
    bool stag;
    int u, issue;
    std::vector<emac_bucket *> bk;
    int nb;
    std::vector<float> us;
  };
  std::vector<V> vs;
  vs.push_back({"seq_u4_i1", 0, false, 4, 1, {}, 0, {}});
  vs.push_back({"seq_u4_i5", 0, false, 4, 5, {}, 0, {}});
  vs.push_back({"seq_u2_i1", 0, false, 2, 1, {}, 0, {}});
  vs.push_back({"seq_u2_i5", 0, false, 2, 5, {}, 0, {}});
  for (long kib : {256L})
    if (kib * 1024 / 16 <= C && C % (kib * 1024 / 16) == 0)
      vs.push_back({"il" + std::to_string(kib) + "K_u4_i5", kib * 1024 / 16, false, 4, 5, {}, 0, {}});
  vs.push_back({"stag_u4_i5", 0, true, 4, 5, {}, 0, {}});
  for (auto &v : vs)
    for (int i = 0; i < nsets; i++) v.bk.push_back(make_buckets(v.stag ? stag[i] : plain[i], C, v.part, v.u, &v.nb));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  emac_codes codes;
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = R;
  CHECK(hipDeviceSynchronize());
  auto run = [&](const V &v, int set) {
    const long TILE = 256L * v.u, ntiles = R * C / TILE, tpb = v.part ? v.part / TILE : C / TILE;
    const dim3 g((unsigned)std::min<long>(ntiles, 8192));
#define NO_K(uu, ii)                                                                                               \
  if (v.u == uu && v.issue == ii)                                                                                  \
    hipLaunchKernelGGL((emac::fold_kernel<float, EMAC_SUM, R, uu, 0, R, ii>), g, dim3(256), 0, s, v.bk[set], v.nb, \
                       ntiles, tpb, 1, codes, (const unsigned *)nullptr, R);
    NO_K(4, 1) NO_K(4, 5) NO_K(2, 1) NO_K(2, 5)
#undef NO_K
  };
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int k = 0;
  for (auto &v : vs)
    for (int i = 0; i < 2; i++) run(v, (k++) % nsets);
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
  printf("node fold order: %d ranks x %ld MiB, %d sets, %d rounds x %d launches (median us, GB/s of %.0f MB)\n", R,
         mib, nsets, rounds, per, bytes / 1e6);
  for (auto &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-8s %9.2f us  %7.1f GB/s  %.3f of 8 TB/s  (min %.2f max %.2f)\n", v.name.c_str(), med,
           bytes / (med * 1e-6) / 1e9, bytes / (med * 1e-6) / 8e12, v.us.front(), v.us.back());
  }
  return 0;
}
