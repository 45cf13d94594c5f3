// fold.hip -- CDNA4 (gfx950) kernels of the bucket-reduction hot path + the HIP runtime ABI.
//
// Replaces gpu_copy_reduce_kernel<T> (reference src/gpu/cuda_core.cu:50-86) and its C-ABI
// (cuda_core.cu:7-106, include/gpu/gpu_core.h:11-22).
//
// The reference kernel walks a per-element descriptor chain in global memory (integer / and %
// per element), reloads and re-stores dst once per SREDUCE line, and writes each fan-out copy
// in a separate launch. Here one launch covers every owner chunk ("bucket") of a plan:
//   * each lane owns 16-byte vectors (dwordx4) of a chunk, U vectors per source in flight;
//   * all R leaf sources are loaded once into VGPRs, then folded in registers in the exact
//     order the reference's SMEMCPY + SREDUCE lines apply them (plan.c's fold tree replayed
//     through per-leaf level codes: a left fold per recursive-halving step, nested);
//   * the result is stored once per destination (fused copy-out fan-out), never re-read.
// HBM traffic per bucket is therefore R reads + D writes of the chunk, the algorithmic
// minimum; the element-wise add is VALU work hidden under the loads (no MFMA: there is no
// contraction here). Integer sums are computed in unsigned arithmetic (two's complement wrap,
// bit-identical to the reference's x86 behaviour without signed-overflow UB); float/double
// keep IEEE round-to-nearest with denormals (no fast-math, no FTZ flags at build time).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "gpu.h"

namespace {

template <typename T> struct Lane;
template <> struct Lane<float> {
  typedef float S;
  typedef float V __attribute__((ext_vector_type(4)));
};
template <> struct Lane<double> {
  typedef double S;
  typedef double V __attribute__((ext_vector_type(2)));
};
template <> struct Lane<int> {
  typedef unsigned int S;
  typedef unsigned int V __attribute__((ext_vector_type(4)));
};
template <> struct Lane<long> {
  typedef unsigned long S;
  typedef unsigned long V __attribute__((ext_vector_type(2)));
};

constexpr int kMaxLevels = 4;  // 16 leaves with radix >= 2

constexpr int pick_unroll(int nsrc) { return nsrc <= 4 ? 4 : (nsrc <= 8 ? 2 : 1); }

// a multi-level tree needs a composite leaf count (every radix >= 2)
constexpr bool can_tree(int n) {
  for (int d = 2; d < n; ++d)
    if (n % d == 0) return true;
  return false;
}

// Replay the fold tree over the leaf values x[0..N) (leaf order of plan.c).
// Linear form (one reduce-scatter radix): ((x0 + x1) + x2) + ...
// Tree form: nested left folds, level l accumulates the completed level-(l-1) partials.
template <int N, bool TREE, typename X>
__device__ __forceinline__ X fold_leaves(const X (&x)[N], const emac_codes &c) {
  if constexpr (!TREE) {
    X acc = x[0];
#pragma unroll
    for (int t = 1; t < N; ++t) acc = acc + x[t];
    return acc;
  } else {
    X cur = x[0];
    X acc[kMaxLevels] = {cur, cur, cur, cur};
#pragma unroll
    for (int t = 0; t < N; ++t) {
      cur = x[t];
#pragma unroll
      for (int l = 0; l < kMaxLevels; ++l) {
        if (l < c.nlev) {  // wave-uniform
          // level l takes a value at leaf t iff levels 0..l-1 all completed at t
          if (l == 0 || c.close[t] >= l) acc[l] = ((c.first[t] >> l) & 1) ? cur : acc[l] + cur;
          cur = acc[l];
        }
      }
    }
    return cur;  // == acc[nlev-1]: the last leaf closes every level
  }
}

template <typename T, int N, bool TREE>
__device__ __forceinline__ void fold_scalar_element(const emac_bucket *b, long e, const emac_codes &c) {
  typedef typename Lane<T>::S S;
  S x[N];
#pragma unroll
  for (int s = 0; s < N; ++s) x[s] = static_cast<const S *>(b->src[s])[e];
  const S r = fold_leaves<N, TREE>(x, c);
  const int nd = b->ndst;
  for (int d = 0; d < nd; ++d) static_cast<S *>(b->dst[d])[e] = r;
}

template <typename T, int N, int U, bool TREE, bool FULL>
__device__ __forceinline__ void fold_vectors(const emac_bucket *b, long v0, const emac_codes &c) {
  typedef typename Lane<T>::S S;
  typedef typename Lane<T>::V V;
  const long head = b->head, nvec = b->nvec;
  V x[U][N];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long v = v0 + (long)u * EMAC_BLOCK;
#pragma unroll
    for (int s = 0; s < N; ++s) {
      const V *p = reinterpret_cast<const V *>(static_cast<const S *>(b->src[s]) + head);
      if (FULL || v < nvec) x[u][s] = p[v];
    }
  }
  V r[U];
#pragma unroll
  for (int u = 0; u < U; ++u) r[u] = fold_leaves<N, TREE>(x[u], c);
  const int nd = b->ndst;
  for (int d = 0; d < nd; ++d) {
    V *q = reinterpret_cast<V *>(static_cast<S *>(b->dst[d]) + head);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long v = v0 + (long)u * EMAC_BLOCK;
      if (FULL || v < nvec) q[v] = r[u];
    }
  }
}

// One workgroup per tile (grid-stride). A tile is EMAC_BLOCK*U consecutive 16-byte vectors of
// one bucket; tile 0 of a bucket also folds the unaligned head/tail elements.
template <typename T, int N, bool TREE>
__global__ __launch_bounds__(EMAC_BLOCK) void fold_kernel(const emac_bucket *__restrict__ bk, int nb,
                                                          long ntiles, emac_codes codes) {
  constexpr int U = pick_unroll(N);
  constexpr long TILE = (long)EMAC_BLOCK * U;
  constexpr long EPV = 16 / sizeof(typename Lane<T>::S);
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    int lo = 0, hi = nb - 1;  // last bucket whose first tile is <= tile (wave-uniform)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (bk[mid].tile0 <= tile)
        lo = mid;
      else
        hi = mid - 1;
    }
    const emac_bucket *b = bk + lo;
    const long t = tile - b->tile0;
    if (b->scalar) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long e = t * TILE + (long)u * EMAC_BLOCK + threadIdx.x;
        if (e < b->nvec) fold_scalar_element<T, N, TREE>(b, e, codes);
      }
      continue;
    }
    if (t == 0) {
      const long nsc = b->head + b->tail;
      if ((long)threadIdx.x < nsc) {
        const long e = (long)threadIdx.x < b->head ? (long)threadIdx.x
                                                   : b->head + b->nvec * EPV + ((long)threadIdx.x - b->head);
        fold_scalar_element<T, N, TREE>(b, e, codes);
      }
    }
    const long v0 = t * TILE + threadIdx.x;
    if ((t + 1) * TILE <= b->nvec)
      fold_vectors<T, N, U, TREE, true>(b, v0, codes);
    else
      fold_vectors<T, N, U, TREE, false>(b, v0, codes);
  }
}

template <typename T, int N>
int launch_n(bool tree, const emac_codes *codes, const emac_bucket *b, int nb, long ntiles,
             hipStream_t stream) {
  const long grid = ntiles < 8192 ? ntiles : 8192;
  if (grid <= 0) return 0;
  if constexpr (can_tree(N)) {
    if (tree) {
      hipLaunchKernelGGL((fold_kernel<T, N, true>), dim3((unsigned)grid), dim3(EMAC_BLOCK), 0, stream, b, nb,
                         ntiles, *codes);
      return hipGetLastError() == hipSuccess ? 0 : EMAC_ERR_DEVICE;
    }
  }
  hipLaunchKernelGGL((fold_kernel<T, N, false>), dim3((unsigned)grid), dim3(EMAC_BLOCK), 0, stream, b, nb,
                     ntiles, *codes);
  return hipGetLastError() == hipSuccess ? 0 : EMAC_ERR_DEVICE;
}

template <typename T>
int launch_t(int nsrc, bool tree, const emac_codes *c, const emac_bucket *b, int nb, long ntiles, hipStream_t s) {
  switch (nsrc) {
  case 1: return launch_n<T, 1>(tree, c, b, nb, ntiles, s);
  case 2: return launch_n<T, 2>(tree, c, b, nb, ntiles, s);
  case 3: return launch_n<T, 3>(tree, c, b, nb, ntiles, s);
  case 4: return launch_n<T, 4>(tree, c, b, nb, ntiles, s);
  case 5: return launch_n<T, 5>(tree, c, b, nb, ntiles, s);
  case 6: return launch_n<T, 6>(tree, c, b, nb, ntiles, s);
  case 7: return launch_n<T, 7>(tree, c, b, nb, ntiles, s);
  case 8: return launch_n<T, 8>(tree, c, b, nb, ntiles, s);
  case 9: return launch_n<T, 9>(tree, c, b, nb, ntiles, s);
  case 10: return launch_n<T, 10>(tree, c, b, nb, ntiles, s);
  case 11: return launch_n<T, 11>(tree, c, b, nb, ntiles, s);
  case 12: return launch_n<T, 12>(tree, c, b, nb, ntiles, s);
  case 13: return launch_n<T, 13>(tree, c, b, nb, ntiles, s);
  case 14: return launch_n<T, 14>(tree, c, b, nb, ntiles, s);
  case 15: return launch_n<T, 15>(tree, c, b, nb, ntiles, s);
  case 16: return launch_n<T, 16>(tree, c, b, nb, ntiles, s);
  }
  return EMAC_ERR_UNSUPPORTED;
}

inline int ok(hipError_t e) { return e == hipSuccess ? 0 : EMAC_ERR_DEVICE; }

}  // namespace

extern "C" {

long emac_gpu_tile_vectors(int dtype, int nsrc) {
  (void)dtype;
  return (long)EMAC_BLOCK * pick_unroll(nsrc);
}

int emac_gpu_fold(int dtype, int op, int nsrc, const emac_codes *codes, const emac_bucket *d_buckets, int nb,
                  long ntiles, void *stream) {
  const bool tree = codes->nlev > 1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (op != EMAC_SUM) return EMAC_ERR_UNSUPPORTED;
  if (nb <= 0 || ntiles <= 0) return 0;
  if (codes->nlev > kMaxLevels) return EMAC_ERR_UNSUPPORTED;
  switch (dtype) {
  case EMAC_FLOAT: return launch_t<float>(nsrc, tree, codes, d_buckets, nb, ntiles, s);
  case EMAC_DOUBLE: return launch_t<double>(nsrc, tree, codes, d_buckets, nb, ntiles, s);
  case EMAC_INT: return launch_t<int>(nsrc, tree, codes, d_buckets, nb, ntiles, s);
  case EMAC_LONG: return launch_t<long>(nsrc, tree, codes, d_buckets, nb, ntiles, s);
  }
  return EMAC_ERR_ARG;
}

int emac_gpu_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
int emac_gpu_get_device(int *dev) { return ok(hipGetDevice(dev)); }
int emac_gpu_set_device(int dev) { return ok(hipSetDevice(dev)); }
int emac_gpu_malloc(void **p, size_t bytes) {
  *p = nullptr;
  if (!bytes) return 0;
  return hipMalloc(p, bytes) == hipSuccess ? 0 : EMAC_ERR_MALLOC;
}
int emac_gpu_free(void *p) { return p ? ok(hipFree(p)) : 0; }
int emac_gpu_memcpy(void *dst, const void *src, size_t bytes) {
  return bytes ? ok(hipMemcpy(dst, src, bytes, hipMemcpyDefault)) : 0;
}
int emac_gpu_memcpy_async(void *dst, const void *src, size_t bytes, void *stream) {
  return bytes ? ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, static_cast<hipStream_t>(stream))) : 0;
}
int emac_gpu_memset_async(void *dst, int v, size_t bytes, void *stream) {
  return bytes ? ok(hipMemsetAsync(dst, v, bytes, static_cast<hipStream_t>(stream))) : 0;
}
int emac_gpu_is_device_pointer(const void *p) {
  hipPointerAttribute_t a;
  if (!p) return 0;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // unregistered host memory: clear the sticky error
    return 0;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}
int emac_gpu_host_register(void *p, size_t bytes) {
  if (!bytes) return 0;
  if (hipHostRegister(p, bytes, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return EMAC_ERR_DEVICE;
  }
  return 0;
}
int emac_gpu_host_unregister(void *p) {
  if (hipHostUnregister(p) != hipSuccess) {
    (void)hipGetLastError();
    return EMAC_ERR_DEVICE;
  }
  return 0;
}
int emac_gpu_stream_create(void **stream) {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return EMAC_ERR_DEVICE;
  *stream = s;
  return 0;
}
int emac_gpu_stream_destroy(void *stream) { return ok(hipStreamDestroy(static_cast<hipStream_t>(stream))); }
int emac_gpu_stream_sync(void *stream) { return ok(hipStreamSynchronize(static_cast<hipStream_t>(stream))); }
int emac_gpu_stream_query(void *stream) {
  hipError_t e = hipStreamQuery(static_cast<hipStream_t>(stream));
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) {
    (void)hipGetLastError();
    return 0;
  }
  return EMAC_ERR_DEVICE;
}
int emac_gpu_device_sync(void) { return ok(hipDeviceSynchronize()); }

}  // extern "C"

// ---- exported device C ABI (include/ext_mpi_amd_gpu.h; reference include/gpu/gpu_core.h) ----
extern "C" {

int ext_mpi_amd_gpu_malloc(void **p, size_t bytes) { return emac_gpu_malloc(p, bytes); }
int ext_mpi_amd_gpu_free(void *p) { return emac_gpu_free(p); }
int ext_mpi_amd_gpu_memcpy_hd(void *dst, const void *src, size_t bytes) {
  return bytes ? ok(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice)) : 0;
}
int ext_mpi_amd_gpu_memcpy_dh(void *dst, const void *src, size_t bytes) {
  return bytes ? ok(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost)) : 0;
}
int ext_mpi_amd_gpu_is_device_pointer(const void *p) { return emac_gpu_is_device_pointer(p); }
int ext_mpi_amd_gpu_synchronize(void) { return emac_gpu_device_sync(); }
int ext_mpi_amd_gpu_device_count(void) { return emac_gpu_device_count(); }
int ext_mpi_amd_gpu_device_of(const void *p) {
  hipPointerAttribute_t a;
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  return (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) ? a.device : -1;
}

// One owner chunk as a one-bucket launch (stream-ordered; the descriptor is staged through a
// small device scratch owned by the call and released after the launch completes).
int ext_mpi_amd_gpu_copy_reduce(int dtype, int op, int nsrc, const void *const *srcs, int ndst, void *const *dsts,
                                long count, void *hip_stream) {
  emac_bucket b;
  emac_codes codes;
  emac_bucket *d = nullptr;
  int tsize = emac_type_size(dtype), rc, i;
  if (tsize < 0 || nsrc < 1 || nsrc > EMAC_MAX_RANKS || ndst < 0 || ndst > EMAC_MAX_RANKS || count < 0)
    return EMAC_ERR_ARG;
  if (!count) return 0;
  memset(&b, 0, sizeof(b));
  memset(&codes, 0, sizeof(codes));
  codes.nlev = 1;
  codes.nleaf = nsrc;
  codes.first[0] = 1;
  codes.close[nsrc - 1] = 1;
  for (i = 0; i < nsrc; i++) b.src[i] = srcs[i];
  for (i = 0; i < ndst; i++) b.dst[i] = dsts[i];
  b.ndst = ndst;
  {
    // same head/vector/tail split as the engine (all pointers must share the 16-byte phase)
    unsigned long mis = (unsigned long)b.src[0] & 15ul;
    long head = (mis % (unsigned long)tsize == 0) ? (long)((16ul - mis) & 15ul) / tsize : -1;
    bool vec = head >= 0;
    if (vec && head > count) head = count;
    for (i = 0; vec && i < nsrc; i++) vec = (((unsigned long)b.src[i] + head * tsize) & 15ul) == 0;
    for (i = 0; vec && i < ndst; i++) vec = (((unsigned long)b.dst[i] + head * tsize) & 15ul) == 0;
    if (vec) {
      b.head = head;
      b.nvec = (count - head) * tsize / 16;
      b.tail = count - head - b.nvec * (16 / tsize);
    } else {
      b.scalar = 1;
      b.nvec = count;
    }
  }
  long tv = emac_gpu_tile_vectors(dtype, nsrc);
  long ntiles = (b.nvec + tv - 1) / tv;
  if (ntiles == 0) ntiles = 1;
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  if (hipMallocAsync((void **)&d, sizeof(b), s) != hipSuccess) return EMAC_ERR_MALLOC;
  if ((rc = ok(hipMemcpyAsync(d, &b, sizeof(b), hipMemcpyHostToDevice, s)))) return rc;
  rc = emac_gpu_fold(dtype, op, nsrc, &codes, d, 1, ntiles, hip_stream);
  (void)hipFreeAsync(d, s);
  if (!rc) rc = ok(hipStreamSynchronize(s));  // the host descriptor lives on this stack frame
  return rc;
}

}  // extern "C"
