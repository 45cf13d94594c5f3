// pcieprobe.hip -- round-3 probe of the host-buffer path's PCIe legs: what rates do the GPU's
// kernels and its DMA engines reach into and out of page-locked host memory, alone and at once?
// (The NODE form with host buffers reads R x S from the host and writes R x S back; bench.py
// measures it at ~39 GB/s each way with the fold kernel doing both over PCIe.)
//   k_rd      kernel: host -> device (nontemporal device stores)
//   k_wr      kernel: device -> host
//   k_rd+k_wr both kernels at once on two streams
//   k_hh      one kernel host -> host (reads and writes over PCIe, like the direct fold)
//   dma_h2d   hipMemcpyAsync host -> device      dma_d2h  device -> host
//   dma_both  both DMA directions at once on two streams
//   dma_h2d+k_wr  DMA in, kernel out, at once
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pcieprobe.hip -o tools/pcieprobe
// Run:   tools/pcieprobe [MiB = 128] [rounds = 5]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ __launch_bounds__(256) void copy_k(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  const long step = (long)gridDim.x * 256 * K;
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
    f4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load(a + i0 + k * 256);
#pragma unroll
    for (int k = 0; k < K; ++k) __builtin_nontemporal_store(v[k], b + i0 + k * 256);
  }
}

int main(int argc, char **argv) {
  const long mib = argc > 1 ? atol(argv[1]) : 128;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  const long bytes = mib << 20, n = bytes / 16;
  f4 *h_in, *h_out, *h_out2, *d_a, *d_b;
  CHECK(hipHostMalloc((void **)&h_in, bytes, hipHostMallocDefault));
  CHECK(hipHostMalloc((void **)&h_out, bytes, hipHostMallocDefault));
  CHECK(hipHostMalloc((void **)&h_out2, bytes, hipHostMallocDefault));
  for (long i = 0; i < n; i++) h_in[i] = f4{(float)i, 1.f, 2.f, 3.f};
  CHECK(hipMalloc(&d_a, bytes));
  CHECK(hipMalloc(&d_b, bytes));
  CHECK(hipMemset(d_a, 0, bytes));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventCreate(&e2));
  struct V {
    std::string name;
    int id, grid;
    double dirs;  // bytes moved over PCIe per run / bytes
    std::vector<float> us;
  };
  std::vector<V> vs = {{"k_rd_g256", 0, 256, 1, {}},      {"k_rd_g1024", 0, 1024, 1, {}},     {"k_rd_g4096", 0, 4096, 1, {}},
                       {"k_wr_g256", 1, 256, 1, {}},      {"k_wr_g1024", 1, 1024, 1, {}},     {"k_wr_g4096", 1, 4096, 1, {}},
                       {"k_rd+k_wr_g1024", 2, 1024, 2, {}}, {"k_hh_g1024", 3, 1024, 2, {}},   {"k_hh_g4096", 3, 4096, 2, {}},
                       {"dma_h2d", 4, 0, 1, {}},          {"dma_d2h", 5, 0, 1, {}},           {"dma_both", 6, 0, 2, {}},
                       {"dma_h2d+k_wr_g1024", 7, 1024, 2, {}}, {"dma_h2d+k_wr_g256", 7, 256, 2, {}}};
  auto run = [&](const V &v) {
    CHECK(hipEventRecord(e0, s1));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    switch (v.id) {
    case 0: hipLaunchKernelGGL((copy_k<4>), dim3(v.grid), dim3(256), 0, s1, h_in, d_a, n); break;
    case 1: hipLaunchKernelGGL((copy_k<4>), dim3(v.grid), dim3(256), 0, s1, d_b, h_out, n); break;
    case 2:
      hipLaunchKernelGGL((copy_k<4>), dim3(v.grid), dim3(256), 0, s1, h_in, d_a, n);
      hipLaunchKernelGGL((copy_k<4>), dim3(v.grid), dim3(256), 0, s2, d_b, h_out, n);
      break;
    case 3: hipLaunchKernelGGL((copy_k<4>), dim3(v.grid), dim3(256), 0, s1, h_in, h_out2, n); break;
    case 4: CHECK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1)); break;
    case 5: CHECK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1)); break;
    case 6:
      CHECK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1));
      CHECK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s2));
      break;
    case 7:
      CHECK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1));
      hipLaunchKernelGGL((copy_k<4>), dim3(v.grid), dim3(256), 0, s2, d_b, h_out, n);
      break;
    }
    CHECK(hipEventRecord(e2, s2));
    CHECK(hipStreamWaitEvent(s1, e2, 0));
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.f;
  };
  for (V &v : vs) run(v);
  for (int r = 0; r < rounds; r++)
    for (V &v : vs) v.us.push_back(run(v));
  printf("PCIe probe: %ld MiB per direction, %d rounds: median min us, GB/s per direction (total)\n", mib, rounds);
  for (V &v : vs) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-22s %9.1f %9.1f  %6.1f GB/s per direction (%6.1f total)\n", v.name.c_str(), med, v.us.front(),
           bytes / med / 1e3, v.dirs * bytes / med / 1e3);
  }
  return 0;
}
