// ceiling.hip -- measured HBM ceilings for bench.py's roofline context (not part of the product
// library; built into tools/libceiling.so by __graft_entry__.build()).
//
//   ceiling_read_glds: a read-only stream through LDS-DMA (global_load_lds_dwordx4, nontemporal):
//                      the best read rate measured on MI355X in round 1 (tools/ldsbench.hip,
//                      ~6.99 TB/s at 4 GiB against ~6.07 TB/s with nt loads into VGPRs).
//   ceiling_read_vgpr: a read-only stream of nontemporal global_load_dwordx4 into VGPRs, K = 4 or 8
//                      vectors per lane in flight (round 3, tools/nodevar.hip,
//                      profiles/r03_nodevar/: 6.85-7.06 TB/s, at or above the LDS-DMA stream on the
//                      same lease); bench.py's read ceiling is the best of the three.
//   ceiling_write:     a write-only stream of nontemporal global_store_dwordx4, K = 4 vectors per lane
//                      (round 3): with the read ceiling it prices a launch that reads and writes as
//                      the sum of its two streams' times (HBM does not read and write at once).
//   ceiling_copy:      a 1:1 copy (1 byte written per byte read: the node-form fold's mix), K = 4
//                      vectors per lane in flight, nontemporal or default-policy accesses.
// Each call enqueues `iters` launches over `bytes` (a multiple of 16 KiB) on `stream`.
#include <hip/hip_runtime.h>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) f4 G4;
typedef __attribute__((address_space(3))) f4 L4;

namespace {

__device__ __forceinline__ void glds16(const f4 *g, L4 *l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)g,
                                   (__attribute__((address_space(3))) void *)l, 16, 0, 2 /* nt */);
}

// each workgroup streams 8 x 4 KiB per pass into LDS and reads one vector back per pass
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

template <int K>
__global__ __launch_bounds__(256) void read_vgpr(const f4 *__restrict__ a, long n, float *out) {
  f4 acc = {0, 0, 0, 0};
  const long step = (long)gridDim.x * 256 * K;
  for (long i0 = (long)blockIdx.x * 256 * K + threadIdx.x; i0 < n; i0 += step) {
    f4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = __builtin_nontemporal_load((const G4 *)a + i0 + k * 256);
#pragma unroll
    for (int k = 0; k < K; ++k) acc += v[k];
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

__global__ __launch_bounds__(256) void write_k4(f4 *__restrict__ b, long n, float v0) {
  const long step = (long)gridDim.x * 256 * 4;
  const f4 v = {v0, v0, v0, v0};
  for (long i0 = (long)blockIdx.x * 256 * 4 + threadIdx.x; i0 < n; i0 += step) {
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(v, (G4 *)b + i0 + k * 256);
  }
}

// a 1:1 copy in phases (the deferred-store order of fold_kernel.hpp fold_deferred): each
// workgroup loads 8 x 256 vectors into LDS, then stores them (tools/nodevar.hip: 6.24 / 6.01 TB/s
// at 128 MiB / 2 GiB against 6.16 / 5.47 for copy_k4 on the same lease)
__global__ __launch_bounds__(256) void copy_phased(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  __shared__ f4 res[8 * 256];
  for (long g0 = (long)blockIdx.x * 2048; g0 < n; g0 += (long)gridDim.x * 2048) {
#pragma unroll
    for (int q = 0; q < 8; ++q) res[q * 256 + threadIdx.x] = __builtin_nontemporal_load((const G4 *)a + g0 + q * 256 + threadIdx.x);
#pragma unroll
    for (int q = 0; q < 8; ++q) __builtin_nontemporal_store(res[q * 256 + threadIdx.x], (G4 *)b + g0 + q * 256 + threadIdx.x);
  }
}

// 1:1 copies, K = 4 vectors per lane in flight, grid-stride: nontemporal (the long streams'
// best) or default-policy (the best below ~64 MiB, where the writes drain through the Infinity
// Cache behind the next launch): tools/schedbench.hip, profiles/r03_schedbench_*.txt
template <bool NT>
__global__ __launch_bounds__(256) void copy_k4(const f4 *__restrict__ a, f4 *__restrict__ b, long n) {
  const long step = (long)gridDim.x * 256 * 4;
  for (long i0 = (long)blockIdx.x * 256 * 4 + threadIdx.x; i0 < n; i0 += step) {
    f4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = NT ? __builtin_nontemporal_load((const G4 *)a + i0 + k * 256) : ((const G4 *)a)[i0 + k * 256];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (NT)
        __builtin_nontemporal_store(v[k], (G4 *)b + i0 + k * 256);
      else
        ((G4 *)b)[i0 + k * 256] = v[k];
    }
  }
}

}  // namespace

extern "C" {

int ceiling_read_glds(const void *buf, long bytes, int iters, float *sink, void *stream) {
  const long n = bytes / 16;
  if (n % (256 * 8) || iters < 1) return -3;
  for (int i = 0; i < iters; i++)
    hipLaunchKernelGGL(read_glds, dim3(2048), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const f4 *>(buf), n,
                       sink);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* k = 4 or 8 vectors per lane in flight */
int ceiling_read_vgpr(const void *buf, long bytes, int iters, int k, float *sink, void *stream) {
  const long n = bytes / 16;
  if (n % (256 * 8) || iters < 1 || (k != 4 && k != 8)) return -3;
  for (int i = 0; i < iters; i++) {
    if (k == 4)
      hipLaunchKernelGGL(read_vgpr<4>, dim3(4096), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const f4 *>(buf), n,
                         sink);
    else
      hipLaunchKernelGGL(read_vgpr<8>, dim3(2048), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const f4 *>(buf), n,
                         sink);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

int ceiling_write(void *buf, long bytes, int iters, void *stream) {
  const long n = bytes / 16;
  if (n % 1024 || iters < 1) return -3;
  for (int i = 0; i < iters; i++)
    hipLaunchKernelGGL(write_k4, dim3(4096), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<f4 *>(buf), n, 1.0f);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* variant 0: nontemporal, 1: default policy, 2: nontemporal in phases (copy_phased) */
int ceiling_copy(const void *src, void *dst, long bytes, int iters, int variant, void *stream) {
  const long n = bytes / 16;
  if (n % 2048 || iters < 1) return -3;
  for (int i = 0; i < iters; i++) {
    if (variant == 2) {
      const long groups = n / 2048;
      hipLaunchKernelGGL(copy_phased, dim3((unsigned)(groups < (1L << 20) ? groups : (1L << 20))), dim3(256), 0,
                         static_cast<hipStream_t>(stream), static_cast<const f4 *>(src), static_cast<f4 *>(dst), n);
    } else if (variant == 0)
      hipLaunchKernelGGL(copy_k4<true>, dim3(4096), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const f4 *>(src),
                         static_cast<f4 *>(dst), n);
    else
      hipLaunchKernelGGL(copy_k4<false>, dim3(4096), dim3(256), 0, static_cast<hipStream_t>(stream), static_cast<const f4 *>(src),
                         static_cast<f4 *>(dst), n);
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}

/* Device memory with hipExtMallocWithFlags flags (bench.py --alloc contig: hipDeviceMallocContiguous,
   physically contiguous, A/B of the translation cost against plain hipMalloc) */
int ceiling_malloc(void **p, size_t bytes, unsigned flags) {
  return hipExtMallocWithFlags(p, bytes, flags) == hipSuccess ? 0 : -1;
}
int ceiling_free(void *p) { return hipFree(p) == hipSuccess ? 0 : -5; }

/* A stream gate for bench.py's timed regions: the stream waits (hipStreamWaitValue32 on a pinned
   host word) until the host opens the gate, so the work enqueued behind it -- the timed region's
   start event and its first launches -- begins only once the host is ahead of the GPU; the timing
   events then hold the kernels and their gaps, not the host's submission latency. */
void *ceiling_gate_arm(void *stream) {
  unsigned *flag = nullptr;
  if (hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return nullptr;
  *flag = 0;
  if (hipStreamWaitValue32(static_cast<hipStream_t>(stream), flag, 1, hipStreamWaitValueGte, 0xFFFFFFFFu) != hipSuccess) {
    (void)hipHostFree(flag);
    return nullptr;
  }
  return flag;
}

void ceiling_gate_open(void *gate) {
  if (!gate) return;
  __atomic_store_n(static_cast<unsigned *>(gate), 1u, __ATOMIC_SEQ_CST);
}

void ceiling_gate_free(void *gate) {
  if (gate) (void)hipHostFree(gate);
}

/* Timing events without the system-scope fence a default event record carries (bench.py's
   per-launch times: the fence would sit between the launches it brackets and change how they run) */
void *ceiling_event_create(void) {
  hipEvent_t e = nullptr;
  return hipEventCreateWithFlags(&e, hipEventDisableSystemFence) == hipSuccess ? (void *)e : nullptr;
}
int ceiling_event_record(void *ev, void *stream) {
  return hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(stream)) == hipSuccess ? 0 : -5;
}
int ceiling_event_ms(void *a, void *b, float *ms) {
  if (hipEventSynchronize(static_cast<hipEvent_t>(b)) != hipSuccess) return -5;
  return hipEventElapsedTime(ms, static_cast<hipEvent_t>(a), static_cast<hipEvent_t>(b)) == hipSuccess ? 0 : -5;
}
void ceiling_event_destroy(void *ev) {
  if (ev) (void)hipEventDestroy(static_cast<hipEvent_t>(ev));
}

}  // extern "C"
