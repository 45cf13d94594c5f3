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
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "gpu.h"
#include "ipc_sync.hpp"

namespace emac {

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

// ISSUE bit 8: peer-mapped (IPC) launch. Leaves may live in another GPU's HBM and results are
// stored into other GPUs' receive buffers, so every access is system-coherent: 16-byte buffer
// loads / stores with sc0 sc1 (cache policy 17: no stale L2 line is ever returned, stores
// write through to the owner's memory). This is what lets the node barriers around the fold
// get away with a single fence each (ipc.hip).
constexpr int kRemote = 256;
constexpr int kSysCoherent = 17;  // sc0 | sc1
// ISSUE bits 9 / 10: default-policy (allocating) stores / loads instead of nontemporal ones. A
// launch whose bytes fit beside the 256 MiB Infinity Cache leaves its results there to drain to
// HBM behind the next launch; nontemporal accesses win on the long streams (tools/pipebench.hip).
constexpr int kPlainStore = 512;
constexpr int kPlainLoad = 1024;
// ISSUE bit 14: stores as 16-byte buffer stores at device scope, nontemporal (cache policy sc1 nt):
// each store is written through the XCD's L2 instead of waiting there as a dirty line for the
// launch's closing write-back. The best of eight store policies in tools/storepol.hip on two
// leases (1-5 % over the default-scope nontemporal store at 16-256 MiB per rank); in the library's
// own launch (U 4 burst, bench.py --schedules) 0.7-1 % faster at 64 and 256 MiB per rank, no gain
// at 16 MiB and below (profiles/r04/storepol/). Offered to the tuner for large node fan-outs,
// with buffer loads (kBufLoad below; engine_tune.c).
constexpr int kDevStore = 1 << 14;
constexpr int kDevStreaming = 18;  // sc1 | nt
// ISSUE bit 15: leaf loads as 16-byte buffer loads (nontemporal, a buffer resource per leaf tile)
// instead of global loads with an SGPR base: the same bytes and cache policy, another address
// path. tools/loadpol.hip: 1-4 % faster under every nontemporal policy on the node fan-out and the
// local fold; in the library's own launch (bench.py --schedules, two passes,
// profiles/r04/bufload/) (U 4, staggered) 0.7-1.2 % faster at 16 / 256 MiB per rank and 4.5 % at
// configs[2]'s 4 MiB, with device-scope stores 0.6 % at 256 MiB, no gain for the other schedules
// or the local fold. The tuner's (U 4, staggered) and device-scope candidates of the node fan-outs
// of 4 and 8 ranks use them, and a (U 4, staggered) buffer-load candidate of the local fold of 4
// or 8 leaves (47.1-47.8 against 47.9 us for its kept LDS groups at 8 x 32 MiB, three passes,
// profiles/r04/bufload/local_*.json) (engine_tune.c).
constexpr int kBufLoad = 1 << 15;
// ISSUE bit 17: stores system-coherent write-through (cache policy sc0 sc1), loads as the other bits
// say: the fused node join's copy-in (join_fused.hip), whose partial is read by peers and by other
// XCDs inside the same launch, after a flag rather than a kernel boundary.
constexpr int kSysStore = 1 << 17;
constexpr int kStreaming = 2;  // nt
typedef unsigned int U32x4 __attribute__((ext_vector_type(4)));

template <typename V>
__device__ __forceinline__ V sys_load16(const void *tile_base, unsigned byte_off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(tile_base), 0, 0x7FFFFFF0, 0x00020000);
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kSysCoherent));
}
template <typename V>
__device__ __forceinline__ void sys_store16(void *tile_base, unsigned byte_off, V v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(tile_base, 0, 0x7FFFFFF0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U32x4, v), r, byte_off, 0, kSysCoherent);
}
template <typename V>
__device__ __forceinline__ V nt_load16(const void *tile_base, unsigned byte_off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(tile_base), 0, 0x7FFFFFF0, 0x00020000);
  return __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kStreaming));
}
template <typename V>
__device__ __forceinline__ void dev_store16(void *tile_base, unsigned byte_off, V v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(tile_base, 0, 0x7FFFFFF0, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(U32x4, v), r, byte_off, 0, kDevStreaming);
}

// The element operation. SUM: a + b (integers in unsigned arithmetic). MIN / MAX as the
// reference's CPU reduction (src/mpi/ext_mpi_native_exec.c:240-318): the accumulator p1 takes
// the incoming p2 iff p2 < p1 (MIN) / p2 > p1 (MAX), compared in the element's own signed /
// IEEE type -- a compare and select, not v_min/v_max, so NaN and signed-zero outcomes follow
// the same order-dependent rule. X is a scalar or a 16-byte vector of T's lane type.
template <int OP, typename T, typename X>
__device__ __forceinline__ X combine(X acc, X x) {
  if constexpr (OP == EMAC_SUM) {
    return acc + x;
  } else {
    constexpr int L = sizeof(X) / sizeof(typename Lane<T>::S);
    if constexpr (L == 1) {
      const T a = (T)acc, b = (T)x;
      return (OP == EMAC_MIN ? b < a : b > a) ? x : acc;
    } else {
      X r = acc;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const T a = (T)acc[i], b = (T)x[i];
        if (OP == EMAC_MIN ? b < a : b > a) r[i] = x[i];
      }
      return r;
    }
  }
}

// a multi-level tree needs a composite leaf count (every radix >= 2)
constexpr bool can_tree(int n) {
  for (int d = 2; d < n; ++d)
    if (n % d == 0) return true;
  return false;
}

// Fold-tree shape as a template parameter CH:
//   0   linear: one reduce-scatter radix, ((x0 + x1) + x2) + ...
//   1   multi-level tree replayed from the plan's runtime level codes (any radix chain)
//   >1  a radix chain known at compile time, packed 5 bits per level, level 0 (the fastest
//       leaf digit, the first reduce-scatter radix of the copy-in string) lowest: the same nested
//       left folds as the runtime codes, but straight-line adds (plan.c build_codes)
constexpr int chain(int r0, int r1, int r2 = 0, int r3 = 0) { return r0 | r1 << 5 | r2 << 10 | r3 << 15; }
constexpr int ch_levels(int ch) { return ch == 0 ? 0 : 1 + ch_levels(ch >> 5); }
constexpr int ch_rad(int ch, int l) { return (ch >> (5 * l)) & 31; }
constexpr int ch_group(int ch, int l) { return l < 0 ? 1 : ch_rad(ch, l) * ch_group(ch, l - 1); }  // leaves per level-l group

// value of the level-L group of chain CH starting at leaf BASE: its first level-(L-1) partial, then
// the others in order (J = 1 .. radix - 1), each combined into the accumulator from the right
template <int OP, typename T, int CH, int L, int BASE, int J, typename X, int N>
__device__ __forceinline__ X chain_rest(const X (&x)[N], X acc);
template <int OP, typename T, int CH, int L, int BASE, typename X, int N>
__device__ __forceinline__ X chain_group(const X (&x)[N]) {
  if constexpr (L < 0) {
    return x[BASE];
  } else {
    return chain_rest<OP, T, CH, L, BASE, 1>(x, chain_group<OP, T, CH, L - 1, BASE>(x));
  }
}
template <int OP, typename T, int CH, int L, int BASE, int J, typename X, int N>
__device__ __forceinline__ X chain_rest(const X (&x)[N], X acc) {
  if constexpr (J == ch_rad(CH, L)) {
    return acc;
  } else {
    constexpr int SUB = ch_group(CH, L - 1);
    return chain_rest<OP, T, CH, L, BASE, J + 1>(x, combine<OP, T>(acc, chain_group<OP, T, CH, L - 1, BASE + J * SUB>(x)));
  }
}

// Replay the fold tree over the leaf values x[0..N) (leaf order of plan.c).
template <int OP, typename T, int N, int CH, typename X>
__device__ __forceinline__ X fold_leaves(const X (&x)[N], const emac_codes &c) {
  if constexpr (CH == 0) {
    X acc = x[0];
#pragma unroll
    for (int t = 1; t < N; ++t) acc = combine<OP, T>(acc, x[t]);
    return acc;
  } else if constexpr (CH > 1) {
    static_assert(ch_group(CH, ch_levels(CH) - 1) == N, "chain does not span the leaves");
    return chain_group<OP, T, CH, ch_levels(CH) - 1, 0>(x);
  } else {
    // runtime codes: level l accumulates the completed level-(l-1) partials
    X cur = x[0];
    X acc[kMaxLevels] = {cur, cur, cur, cur};
#pragma unroll
    for (int t = 0; t < N; ++t) {
      cur = x[t];
#pragma unroll
      for (int l = 0; l < kMaxLevels; ++l) {
        if (l < c.nlev) {  // wave-uniform
          // level l takes a value at leaf t iff levels 0..l-1 all completed at t
          if (l == 0 || c.close[t] >= l) acc[l] = ((c.first[t] >> l) & 1) ? cur : combine<OP, T>(acc[l], cur);
          cur = acc[l];
        }
      }
    }
    return cur;  // == acc[nlev-1]: the last leaf closes every level
  }
}

// D = fan-out width, a compile-time constant: N for the node form (every rank's receive
// buffer), 1 for the communicator form. All destination pointers are then loaded up front.
template <typename T, int OP, int N, int CH, int D, bool REMOTE = false>
__device__ __forceinline__ void fold_scalar_element(const emac_bucket *b, long e, const emac_codes &c) {
  typedef typename Lane<T>::S S;
  const long k = e - b->head;  // bucket pointers sit at element `head`
  S x[N];
#pragma unroll
  for (int s = 0; s < N; ++s) {
    const S *p = static_cast<const S *>(b->src[s]) + k;
    if constexpr (REMOTE)
      x[s] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      x[s] = *p;
  }
  const S r = fold_leaves<OP, T, N, CH>(x, c);
#pragma unroll
  for (int d = 0; d < D; ++d) {
    S *p = static_cast<S *>(b->dst[d]) + k;
    if constexpr (REMOTE)
      __hip_atomic_store(p, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      *p = r;
  }
}

// Loads are nontemporal (each leaf byte is read exactly once; keeping it out of L2/MALL leaves
// room for the concurrent stream), stores too (results are not re-read by this launch).
// Measured +12 % at 16 MiB x 8 ranks over plain loads/stores (tools/foldbench.hip).
// All leaf / destination pointers of the bucket are read into scalar registers once, before
// any load is issued, and used as global (address space 1) bases: the loads become
// `global_load_dwordx4 v, v_off, s_base nt` issued back to back, instead of flat loads each
// waiting on its own descriptor read.
// ISSUE (load issue schedule, measured in tools/ldsbench.hip): bit 0 = source-major order
// (every vector of leaf 0, then leaf 1, ...) instead of vector-major; bits 1.. = s_sleep after
// every 4 loads (0 = back-to-back burst).
// Loads and folds one tile: r[u] = the fold of every leaf's vector u of the tile.
// BS: the workgroup's lanes (a tile is BS * U vectors; EMAC_BLOCK but for the fused node join's
// 1024-lane workgroups, join_fused.hip)
template <typename T, int OP, int N, int U, int CH, bool FULL, int ISSUE, int BS = EMAC_BLOCK>
__device__ __forceinline__ void load_fold(const emac_bucket *b, long tile_base, long nvec, const emac_codes &c,
                                          typename Lane<T>::V (&r)[U]) {
  typedef typename Lane<T>::V V;
  typedef __attribute__((address_space(1))) V GV;
  constexpr bool SRC_MAJOR = ISSUE & 1;
  constexpr int SLEEP = (ISSUE >> 1) & 127;  // bits 1..7
  constexpr bool REMOTE = ISSUE & kRemote;
  // vectors of this tile still inside the bucket (wave-uniform); lane offsets are 32-bit so
  // every access is `global_*_dwordx4 v, v_off, s_base` with the tile base in SGPRs
  const long left = nvec - tile_base;
  V x[U][N];
  const GV *src[N];
#pragma unroll
  for (int s = 0; s < N; ++s) src[s] = (const GV *)b->src[s] + tile_base;
#pragma unroll
  for (int k = 0; k < N * U; ++k) {
    const int s = SRC_MAJOR ? k / U : k % N, u = SRC_MAJOR ? k % U : k / N;
    const unsigned v = threadIdx.x + (unsigned)(u * BS);
    if constexpr (REMOTE) {
      if (FULL || (long)v < left) x[u][s] = sys_load16<V>((const void *)src[s], v * 16u);
    } else if constexpr ((ISSUE & kPlainLoad) != 0) {
      if (FULL || (long)v < left) x[u][s] = src[s][v];
    } else if constexpr ((ISSUE & kBufLoad) != 0) {
      if (FULL || (long)v < left) x[u][s] = nt_load16<V>((const void *)src[s], v * 16u);
    } else {
      if (FULL || (long)v < left) x[u][s] = __builtin_nontemporal_load(src[s] + v);
    }
    if constexpr (SLEEP > 0) {
      if ((k & 3) == 3 && k + 1 < N * U) __builtin_amdgcn_s_sleep(SLEEP);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) r[u] = fold_leaves<OP, T, N, CH>(x[u], c);
}

// ISSUE bit 19 (with kRemote): no store drain after each tile (fold_vectors); the fused node join
// drains once per segment, before it counts the segment's items (join_fused.hip join_seg)
constexpr int kNoDrain = 1 << 19;

// One 16-byte vector stored under the launch's store policy.
template <typename V, int ISSUE>
__device__ __forceinline__ void store_vec(__attribute__((address_space(1))) V *dst, unsigned v, V r) {
  if constexpr ((ISSUE & (kRemote | kSysStore)) != 0)
    sys_store16<V>((void *)dst, v * 16u, r);
  else if constexpr ((ISSUE & kDevStore) != 0)
    dev_store16<V>((void *)dst, v * 16u, r);
  else if constexpr ((ISSUE & kPlainStore) != 0)
    dst[v] = r;
  else
    __builtin_nontemporal_store(r, dst + v);
}

template <typename T, int OP, int N, int U, int CH, int D, bool FULL, int ISSUE = 1, int BS = EMAC_BLOCK>
__device__ __forceinline__ void fold_vectors(const emac_bucket *b, long tile_base, long nvec, const emac_codes &c,
                                             bool store = true) {
  typedef typename Lane<T>::V V;
  typedef __attribute__((address_space(1))) V GV;
  constexpr bool REMOTE = ISSUE & kRemote;
  const long left = nvec - tile_base;
  V r[U];
  load_fold<T, OP, N, U, CH, FULL, ISSUE, BS>(b, tile_base, nvec, c, r);
  // destination pointers are only needed now: their descriptor read overlaps the loads
  if (!store) return;  // peer-mapped launch whose phase-0 barrier failed (wave-uniform)
#pragma unroll
  for (int d = 0; d < D; ++d) {
    GV *dst = (GV *)b->dst[d] + tile_base;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const unsigned v = threadIdx.x + (unsigned)(u * BS);
      if (FULL || (long)v < left) store_vec<V, ISSUE>(dst, v, r[u]);
    }
  }
  // a peer-mapped launch's stores are acknowledged by the owners' memory before the wave ends,
  // so the barrier launch after it can signal without a release fence (kNoDrain: the caller
  // drains once for many items, join_fused.hip)
  if constexpr (REMOTE && (ISSUE & kNoDrain) == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ISSUE bits 11-12 (kDeferShift): deferred stores. A workgroup takes KB = 2^k consecutive tiles
// of one bucket, folds them one after the other into LDS, then stores all KB tiles to every
// destination in one burst. The workgroups, started together, then alternate between phases of
// loads and phases of stores instead of mixing both all the time: fewer read/write turnarounds
// at the HBM (tools/nodevar.hip, profiles/r03_nodevar/: the local fold 8 x 32 MiB -> 1 at 0.79-0.80
// of 8 TB/s against 0.76-0.77 for the per-tile loop, 2-4 % at every size measured back to back; the
// node fan-out 2 % faster at 16 MiB per rank on one lease, slower on others, and behind the
// staggered per-tile schedule in the bench's steady state, profiles/r03_tune/force_ab.txt). Each
// lane reads back only the LDS slots it wrote, so no barrier is needed. Offered to the per-handle
// tuner (engine.c emac_tune); the fold order -- and so every bit -- is the per-tile loop's.
constexpr int kDeferShift = 11;
constexpr int defer_tiles(int issue) { return ((issue >> kDeferShift) & 3) ? 1 << ((issue >> kDeferShift) & 3) : 1; }
constexpr int defer(int kb) { return (kb == 2 ? 1 : kb == 4 ? 2 : kb == 8 ? 3 : 0) << kDeferShift; }
// ISSUE bit 13 (with deferred stores, linear fold only): leaf-major groups. The group's KB * U
// vectors per lane are read leaf after leaf -- each leaf's KB * U KiB per wave back to back -- and
// accumulated in registers in the leaves' order, ((x0 + x1) + x2) + ..., the linear fold's bits;
// no LDS, 80 VGPRs at KB * U = 8 (occupancy 6 against 4). The node fan-out only: 3.5-4.5 % faster
// than the LDS groups per Start in the bench's steady state at 16 MiB per rank
// (profiles/r03_tune/force_ab.txt).
constexpr int kLeafMajor = 1 << 13;

// One group of fold_deferred_kernel: nt (<= KB) consecutive tiles of bucket b from vector gbase. ALL_FULL
// (host-known: every tile of every bucket whole and every group KB tiles) skips the bucket's vector
// count -- a dependent scalar load that would otherwise stand before the group's first leaf load --
// and every guard on nt.
template <typename T, int OP, int N, int U, int CH, int D, int ISSUE, bool ALL_FULL>
__device__ __forceinline__ void fold_group(const emac_bucket *b, long gbase, int nt, const emac_codes &c,
                                           typename Lane<T>::V *res) {
  typedef typename Lane<T>::V V;
  typedef __attribute__((address_space(1))) V GV;
  constexpr int KB = defer_tiles(ISSUE);
  constexpr long TILE = (long)EMAC_BLOCK * U;
  const long nvec = ALL_FULL ? 0 : b->nvec;
#pragma unroll
  for (int j = 0; j < KB; ++j) {
    if (ALL_FULL || j < nt) {
      const long tb = gbase + j * TILE;
      V r[U];
      if (ALL_FULL || tb + TILE <= nvec)
        load_fold<T, OP, N, U, CH, true, ISSUE>(b, tb, nvec, c, r);
      else
        load_fold<T, OP, N, U, CH, false, ISSUE>(b, tb, nvec, c, r);
#pragma unroll
      for (int u = 0; u < U; ++u) res[(j * U + u) * EMAC_BLOCK + threadIdx.x] = r[u];
    }
  }
  const long left = nvec - gbase;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    GV *dst = (GV *)b->dst[d] + gbase;
#pragma unroll
    for (int q = 0; q < KB * U; ++q) {
      const unsigned v = threadIdx.x + (unsigned)(q * EMAC_BLOCK);
      if (ALL_FULL || (q < nt * U && (long)v < left)) store_vec<V, ISSUE>(dst, v, res[q * EMAC_BLOCK + threadIdx.x]);
    }
  }
}

// ISSUE bit 16 (kLmOpenCopy, with kLeafMajor over a compile-time chain): every leaf is loaded into
// registers of its own and a level-0 group's opening leaf is then copied into the group's
// accumulator behind an empty asm statement, instead of being loaded into the accumulator itself.
// It changes the compiler's schedule of the chains' leaf loads (the linear fold does not need it).
// 16 MiB x 8 per Start, forced, one lease (profiles/r05/chains/): -2 -4 44.1 against 47.1 us
// without it, -2 -2 -2 45.5 against 48.2, -4 -2 45.7 against 45.3; the linear fold 44.6. Both forms
// are tuner candidates of the chains' fan-out (engine_tune.c).
constexpr int kLmOpenCopy = 1 << 16;

// Leaf-major groups over a fold tree (kLeafMajor, round 5: any compile-time chain as well as the
// linear fold). The tree's level l has lm_levels(CH, N) levels; level l groups lm_group(CH, N, l)
// consecutive leaves (the linear fold: one level of N). Leaves arrive one after the other, so each
// open level keeps one accumulator per vector: leaf t enters level 0 -- starting it when t opens a
// level-0 group, else combined from the right -- and when t completes a level-(l-1) group that
// partial enters level l the same way. These are chain_group's nested left folds in the same order,
// so the bits are fold_leaves' (the linear fold: ((x0 + x1) + x2) + ...).
constexpr int lm_levels(int ch) { return ch == 0 ? 1 : ch_levels(ch); }
constexpr int lm_group(int ch, int n, int l) { return ch == 0 ? (l < 0 ? 1 : n) : ch_group(ch, l); }

// leaf T has completed the level-(L-1) group it belongs to: that partial enters level L
template <int OP, typename T, int N, int CH, int T_, int L, int Q, typename V>
__device__ __forceinline__ void lm_close(V (&acc)[lm_levels(CH)][Q]) {
  if constexpr (L < lm_levels(CH)) {
    if constexpr ((T_ + 1) % lm_group(CH, N, L - 1) == 0) {
      constexpr bool first = T_ % lm_group(CH, N, L) < lm_group(CH, N, L - 1);
#pragma unroll
      for (int q = 0; q < Q; ++q) acc[L][q] = first ? acc[L - 1][q] : combine<OP, T>(acc[L][q], acc[L - 1][q]);
      lm_close<OP, T, N, CH, T_, L + 1, Q>(acc);
    }
  }
}

// leaves S .. N-1 of the group, read leaf after leaf (each leaf's Q vectors per lane back to back).
// BOUNDED (a group that reaches past its bucket's last vector): every leaf read is a buffer load
// whose resource ends at the bucket's end, so loads past it return 0 instead of needing a guard;
// the code stays straight-line (guarded loads and adds had made the compiler spill the
// accumulators to scratch) and only the stores are guarded.
template <typename T, int OP, int N, int CH, int Q, int ISSUE, bool BOUNDED, int S, typename V>
__device__ __forceinline__ void lm_leaves(const emac_bucket *b, long gbase, unsigned bound, V (&acc)[lm_levels(CH)][Q]) {
  typedef __attribute__((address_space(1))) V GV;
  if constexpr (S < N) {
    constexpr bool opens = S % lm_group(CH, N, 0) == 0;  // leaf S starts a level-0 group
    const GV *src = (const GV *)b->src[S] + gbase;
    V x[Q];
    constexpr bool VIA_X = (ISSUE & kLmOpenCopy) != 0;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const unsigned v = threadIdx.x + (unsigned)(q * EMAC_BLOCK);
      V &dst = opens && !VIA_X ? acc[0][q] : x[q];
      if constexpr (BOUNDED) {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, bound, 0x00020000);
        dst = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(r, v * 16u, 0, kStreaming));
      } else if constexpr ((ISSUE & kBufLoad) != 0) {
        dst = nt_load16<V>((const void *)src, v * 16u);
      } else {
        dst = __builtin_nontemporal_load(src + v);
      }
    }
    if constexpr (!opens) {
#pragma unroll
      for (int q = 0; q < Q; ++q) acc[0][q] = combine<OP, T>(acc[0][q], x[q]);
    } else if constexpr (VIA_X) {
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        acc[0][q] = x[q];
        asm volatile("" : "+v"(acc[0][q]));
      }
    }
    lm_close<OP, T, N, CH, S, 1, Q>(acc);
    lm_leaves<T, OP, N, CH, Q, ISSUE, BOUNDED, S + 1>(b, gbase, bound, acc);
  }
}

// One leaf-major group: vector q of the group is lane vector q * EMAC_BLOCK + lane from gbase (the
// KB tiles of U vectors are contiguous); no LDS.
template <typename T, int OP, int N, int U, int CH, int D, int ISSUE, bool ALL_FULL>
__device__ __forceinline__ void fold_group_leaf(const emac_bucket *b, long gbase, int nt) {
  typedef typename Lane<T>::V V;
  typedef __attribute__((address_space(1))) V GV;
  constexpr int Q = defer_tiles(ISSUE) * U;
  constexpr int LV = lm_levels(CH);
  static_assert(lm_group(CH, N, LV - 1) == N, "the fold tree spans the leaves");
  // vectors of the group inside the bucket (a whole group unless it holds the bucket's last tile)
  const long left = ALL_FULL ? (long)Q * EMAC_BLOCK : b->nvec - gbase;
  V acc[LV][Q];
  if (ALL_FULL || left >= (long)Q * EMAC_BLOCK) {
    lm_leaves<T, OP, N, CH, Q, ISSUE, false, 0>(b, gbase, 0u, acc);
  } else {
    lm_leaves<T, OP, N, CH, Q, ISSUE, true, 0>(b, gbase, (unsigned)(left > 0 ? left * 16 : 0), acc);
  }
  // each group starts its stores at destination (group index mod D), so the groups in flight write
  // all D receive buffers at once rather than each in turn: 0.6-0.9 % faster at 16 MiB per rank,
  // three passes (profiles/r04/leafshape/rotdst_*.json); the same values land in every buffer. (One
  // guarded store loop: a second, unguarded one for whole groups took the partial-group kernels
  // from 112 to 255 VGPRs and the -64 fractions from 46.1 to 49.5 us, profiles/r05/chains/.)
  const int d0 = (int)((unsigned long)gbase / (unsigned long)(Q * EMAC_BLOCK) % (unsigned)D);
#pragma unroll
  for (int dd = 0; dd < D; ++dd) {
    const int d = dd + d0 < D ? dd + d0 : dd + d0 - D;
    GV *dst = (GV *)b->dst[d] + gbase;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const unsigned v = threadIdx.x + (unsigned)(q * EMAC_BLOCK);
      if (ALL_FULL || (long)v < left) store_vec<V, ISSUE>(dst, v, acc[LV - 1][q]);
    }
  }
  (void)nt;
}

// The deferred-store schedule as a kernel of its own, so its code holds nothing of the per-tile
// loop's: equal buckets of tpb tiles, or (MAP, round 5) up to EMAC_GROUP_MAP_MAX buckets of any
// tile counts whose first groups the layout wrote into their tile0 (layout.c): each wave loads
// those starts into its registers once, and a group's bucket is the number of starts at or below it,
// one ballot (the `-k` fractions' few short chunks beside a long one get the leaf-major
// and LDS groups instead of the per-tile loop).
template <typename T, int OP, int N, int U, int CH, int D, int ISSUE, bool ALL_FULL, bool MAP = false>
__device__ __forceinline__ void deferred_body(const emac_bucket *__restrict__ bk, long tpb, long ngroups,
                                              const emac_codes &codes, int nb = 0) {
  typedef typename Lane<T>::V V;
  static_assert(N > 0 && (ISSUE & kRemote) == 0, "deferred stores: compile-time leaves, local memory");
  static_assert((ISSUE & kLeafMajor) == 0 || CH != 1, "leaf-major groups: compile-time fold trees");
  constexpr int KB = defer_tiles(ISSUE);
  constexpr long TILE = (long)EMAC_BLOCK * U;
  constexpr bool LEAF = (ISSUE & kLeafMajor) != 0;
  __shared__ V res[LEAF ? 1 : KB * U * EMAC_BLOCK];
  // groups per bucket (the last one may hold fewer tiles); group counts fit 32 bits (< 2^31 groups
  // of >= 8 KiB), and 32-bit division is a short sequence ahead of the group's first load
  const unsigned gpb = MAP ? 1u : (unsigned)((tpb + KB - 1) / KB);
  // the bucket map in each wave's own registers: lane i holds bucket i's first group (no LDS table,
  // no barrier ahead of the first leaf load)
  unsigned gt = ~0u;
  if constexpr (MAP) {
    static_assert(!ALL_FULL, "bucket-mapped groups check their bucket's end");
    static_assert(EMAC_GROUP_MAP_MAX <= 64, "one lane per bucket of the map");
    const unsigned lane = threadIdx.x & 63u;
    if (lane < (unsigned)nb) gt = (unsigned)bk[lane].tile0;
  }
  for (long g = blockIdx.x; g < ngroups; g += gridDim.x) {
    int bi;
    long t0;
    int nt;
    if constexpr (MAP) {
      bi = __popcll(__ballot(gt <= (unsigned)g)) - 1;  // starts ascend: the last one <= g
      t0 = (g - (long)(unsigned)__builtin_amdgcn_readlane((int)gt, bi)) * KB;
      const long tb = (bk[bi].nvec + TILE - 1) / TILE;  // the bucket's tiles
      nt = tb - t0 < KB ? (int)(tb - t0) : KB;
    } else {
      bi = (int)((unsigned)g / gpb);
      t0 = (g - (long)bi * gpb) * KB;
      nt = tpb - t0 < KB ? (int)(tpb - t0) : KB;  // wave-uniform
    }
    if constexpr (LEAF)
      fold_group_leaf<T, OP, N, U, CH, D, ISSUE, ALL_FULL>(bk + bi, t0 * TILE, nt);
    else
      fold_group<T, OP, N, U, CH, D, ISSUE, ALL_FULL>(bk + bi, t0 * TILE, nt, codes, res);
  }
}

template <typename T, int OP, int N, int U, int CH, int D, int ISSUE, bool ALL_FULL>
__global__ __launch_bounds__(EMAC_BLOCK) void fold_deferred_kernel(const emac_bucket *__restrict__ bk, long tpb,
                                                                   long ngroups, emac_codes codes) {
  deferred_body<T, OP, N, U, CH, D, ISSUE, ALL_FULL>(bk, tpb, ngroups, codes);
}

template <typename T, int OP, int N, int U, int CH, int D, int ISSUE>
__global__ __launch_bounds__(EMAC_BLOCK) void fold_deferred_map_kernel(const emac_bucket *__restrict__ bk, int nb,
                                                                       long ngroups, emac_codes codes) {
  deferred_body<T, OP, N, U, CH, D, ISSUE, false, true>(bk, -1, ngroups, codes, nb);
}

// ---- runtime leaf count (N = 0 in the templates below): MIN / MAX ----
// The reference's CPU reduction also takes MIN and MAX (ext_mpi_native_exec.c:240-318); they are
// off the hot path (its GPU kernel only sums), so they run ONE kernel per element type, operation
// and fan-out form: up to kRtMax leaves read with wave-uniform guards, the plan's runtime level
// codes (nlev 1 for a linear fold), one 16-byte vector per lane and leaf. D = 1: one destination;
// D = 0: `n` destinations (the node form's fan-out).
constexpr int kRtMax = EMAC_MAX_RANKS;

template <int OP, typename T, typename X>
__device__ __forceinline__ X fold_leaves_rt(const X (&x)[kRtMax], int n, const emac_codes &c) {
  X cur = x[0];
  X acc[kMaxLevels] = {cur, cur, cur, cur};
#pragma unroll
  for (int t = 0; t < kRtMax; ++t) {
    if (t < n) {  // wave-uniform
      cur = x[t];
#pragma unroll
      for (int l = 0; l < kMaxLevels; ++l) {
        if (l < c.nlev) {
          if (l == 0 || c.close[t] >= l) acc[l] = ((c.first[t] >> l) & 1) ? cur : combine<OP, T>(acc[l], cur);
          cur = acc[l];
        }
      }
    }
  }
  return cur;
}

template <typename T, int OP, int D, bool REMOTE>
__device__ __forceinline__ void fold_scalar_rt(const emac_bucket *b, long e, const emac_codes &c, int n) {
  typedef typename Lane<T>::S S;
  const long k = e - b->head;
  S x[kRtMax];
#pragma unroll
  for (int s = 0; s < kRtMax; ++s) {
    if (s < n) {
      const S *p = static_cast<const S *>(b->src[s]) + k;
      if constexpr (REMOTE)
        x[s] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        x[s] = *p;
    }
  }
  const S r = fold_leaves_rt<OP, T>(x, n, c);
  const int nd = D ? 1 : n;
#pragma unroll
  for (int d = 0; d < kRtMax; ++d) {
    if (d < nd) {
      S *p = static_cast<S *>(b->dst[d]) + k;
      if constexpr (REMOTE)
        __hip_atomic_store(p, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      else
        *p = r;
    }
  }
}

template <typename T, int OP, int D, bool FULL, bool REMOTE>
__device__ __forceinline__ void fold_vectors_rt(const emac_bucket *b, long tile_base, long nvec, const emac_codes &c,
                                                int n, bool store) {
  typedef typename Lane<T>::V V;
  typedef __attribute__((address_space(1))) V GV;
  const long left = nvec - tile_base;
  const unsigned v = threadIdx.x;
  V x[kRtMax];
#pragma unroll
  for (int s = 0; s < kRtMax; ++s) {
    if (s < n && (FULL || (long)v < left)) {
      const GV *src = (const GV *)b->src[s] + tile_base;
      if constexpr (REMOTE)
        x[s] = sys_load16<V>((const void *)src, v * 16u);
      else
        x[s] = __builtin_nontemporal_load(src + v);
    }
  }
  const V r = fold_leaves_rt<OP, T>(x, n, c);
  if (!store || !(FULL || (long)v < left)) return;
  const int nd = D ? 1 : n;
#pragma unroll
  for (int d = 0; d < kRtMax; ++d) {
    if (d < nd) {
      GV *dst = (GV *)b->dst[d] + tile_base;
      if constexpr (REMOTE)
        sys_store16<V>((void *)dst, v * 16u, r);
      else
        __builtin_nontemporal_store(r, dst + v);
    }
  }
}

// Streaming body: one workgroup per tile (grid-stride); a tile is EMAC_BLOCK*U consecutive
// 16-byte vectors of one bucket. Nothing element-granular runs here (see fold_edge_kernel).
template <typename T, int OP, int N, int U, int CH, int D, int ISSUE = 1>
__global__ __launch_bounds__(EMAC_BLOCK) void fold_kernel(const emac_bucket *__restrict__ bk, int nb,
                                                          long ntiles, long tiles_per_bucket, int all_full,
                                                          emac_codes codes, const unsigned *go, int nrt) {
  constexpr long TILE = (long)EMAC_BLOCK * U;
  static_assert(N > 0 || U == 1, "runtime leaf counts use one vector per lane");
  // peer-mapped launch: the phase-0 barrier's verdict (ipc_sync.hpp); its load is issued ahead of
  // the leaf loads and only waited for before the first store
  bool store = true;
  if constexpr ((ISSUE & kRemote) != 0) store = __hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
  static_assert(defer_tiles(ISSUE) == 1, "deferred stores: fold_deferred_kernel");
  for (long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // bucket of this tile: arithmetic when every bucket has the same tile count (equal chunks:
    // the common case), else the last bucket whose first tile is <= tile (wave-uniform search;
    // each probe is a dependent scalar load, so it is avoided whenever possible)
    int bi;
    long t;
    if (tiles_per_bucket > 0) {
      // tile counts fit 32 bits (< 2^31 tiles of >= 4 KiB); 32-bit division is a short sequence
      bi = (int)((unsigned)tile / (unsigned)tiles_per_bucket);
      t = tile - (long)bi * tiles_per_bucket;
    } else {
      int lo = 0, hi = nb - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (bk[mid].tile0 <= tile)
          lo = mid;
        else
          hi = mid - 1;
      }
      bi = lo;
      t = tile - bk[lo].tile0;
    }
    const emac_bucket *b = bk + bi;
    // all_full (host-known: every bucket a whole number of tiles) skips the dependent read of
    // nvec before the first load of the tile
    if constexpr (N == 0) {
      constexpr bool REMOTE = (ISSUE & kRemote) != 0;
      if (all_full || (t + 1) * TILE <= b->nvec)
        fold_vectors_rt<T, OP, D, true, REMOTE>(b, t * TILE, 0, codes, nrt, store);
      else
        fold_vectors_rt<T, OP, D, false, REMOTE>(b, t * TILE, b->nvec, codes, nrt, store);
      if constexpr (REMOTE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (all_full || (t + 1) * TILE <= b->nvec)
        fold_vectors<T, OP, N, U, CH, D, true, ISSUE>(b, t * TILE, 0, codes, store);
      else
        fold_vectors<T, OP, N, U, CH, D, false, ISSUE>(b, t * TILE, b->nvec, codes, store);
    }
  }
}

// Element-granular work: unaligned heads/tails and misaligned buckets, one workgroup per item.
template <typename T, int OP, int N, int CH, int D, bool REMOTE = false>
__global__ __launch_bounds__(EMAC_BLOCK) void fold_edge_kernel(const emac_bucket *__restrict__ bk,
                                                               const emac_edge *__restrict__ items,
                                                               emac_codes codes, const unsigned *go, int nrt) {
  constexpr long EPV = 16 / sizeof(typename Lane<T>::S);
  if constexpr (REMOTE) {
    if (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) return;
  }
  const emac_edge it = items[blockIdx.x];
  const emac_bucket *b = bk + it.bucket;
  auto one = [&](long e) {
    if constexpr (N == 0)
      fold_scalar_rt<T, OP, D, REMOTE>(b, e, codes, nrt);
    else
      fold_scalar_element<T, OP, N, CH, D, REMOTE>(b, e, codes);
  };
  if (it.mode == 1) {
    for (long e = it.start + threadIdx.x; e < it.start + it.count; e += EMAC_BLOCK) one(e);
  } else {
    const long nsc = b->head + b->tail;
    for (long i = threadIdx.x; i < nsc; i += EMAC_BLOCK) one(i < b->head ? i : b->head + b->nvec * EPV + (i - b->head));
  }
  if constexpr (REMOTE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// A set of buckets of one launch as kernel arguments (the fused kernel runs two: the fold of
// this rank's owner chunks and the pull of every other owner's result).
typedef emac_join_ctl JoinCtl;

struct Work {
  const emac_bucket *b;
  int nb;
  long ntiles, tpb;
  int all_full;
  const emac_edge *edges;
  int nedges;
};

// Every tile and edge item of `w`, grid-strided over the launch's workgroups, with
// system-coherent accesses (fold_vectors REMOTE). N leaves (N = 1: a copy).
template <typename T, int OP, int N, int U, int CH>
__device__ __forceinline__ void run_remote(const Work &w, const emac_codes &codes, int nrt = 0) {
  constexpr int ISSUE = 1 | kRemote;
  constexpr long TILE = (long)EMAC_BLOCK * U;
  constexpr long EPV = 16 / sizeof(typename Lane<T>::S);
  for (long tile = blockIdx.x; tile < w.ntiles; tile += gridDim.x) {
    int bi;
    long t;
    if (w.tpb > 0) {
      bi = (int)((unsigned)tile / (unsigned)w.tpb);
      t = tile - (long)bi * w.tpb;
    } else {
      int lo = 0, hi = w.nb - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (w.b[mid].tile0 <= tile)
          lo = mid;
        else
          hi = mid - 1;
      }
      bi = lo;
      t = tile - w.b[lo].tile0;
    }
    const emac_bucket *b = w.b + bi;
    if constexpr (N == 0) {
      if (w.all_full || (t + 1) * TILE <= b->nvec)
        fold_vectors_rt<T, OP, 1, true, true>(b, t * TILE, 0, codes, nrt, true);
      else
        fold_vectors_rt<T, OP, 1, false, true>(b, t * TILE, b->nvec, codes, nrt, true);
    } else {
      if (w.all_full || (t + 1) * TILE <= b->nvec)
        fold_vectors<T, OP, N, U, CH, 1, true, ISSUE>(b, t * TILE, 0, codes);
      else
        fold_vectors<T, OP, N, U, CH, 1, false, ISSUE>(b, t * TILE, b->nvec, codes);
    }
  }
  for (int item = blockIdx.x; item < w.nedges; item += gridDim.x) {
    const emac_edge it = w.edges[item];
    const emac_bucket *b = w.b + it.bucket;
    auto one = [&](long e) {
      if constexpr (N == 0)
        fold_scalar_rt<T, OP, 1, true>(b, e, codes, nrt);
      else
        fold_scalar_element<T, OP, N, CH, 1, true>(b, e, codes);
    };
    if (it.mode == 1) {
      for (long e = it.start + threadIdx.x; e < it.start + it.count; e += EMAC_BLOCK) one(e);
    } else {
      const long nsc = b->head + b->tail;
      for (long i = threadIdx.x; i < nsc; i += EMAC_BLOCK) one(i < b->head ? i : b->head + b->nvec * EPV + (i - b->head));
    }
  }
}

// The whole peer-mapped Allreduce in ONE launch, for small messages where the kernel boundaries
// of barrier -> fold -> barrier -> pull cost as much as the work (each ≈ 1.5-2 us).
//  phase 0 (ipc_sync.hpp): workgroup 0's first wave signals every peer, the first wave of EVERY
//          workgroup waits for them (a workgroup folds only after it has seen every peer ready);
//  fold:   this rank's owner chunks, leaves loaded from the peers' send buffers, the result
//          stored (write-through) into this rank's own outbox only;
//  phase 1: each workgroup drains its stores and counts itself in arrive[slot]; the last one
//          signals the peers and this rank itself (its own flag: every own chunk has landed);
//          every workgroup waits for every peer's signal and for its own rank's;
//  pull:   every owner's result (this rank's own too) loaded from that owner's outbox and stored
//          into this rank's receive buffer. The receive buffer is only ever written by its own
//          rank: lines of it that this rank's L2s hold stay coherent with what the application
//          reads next (measured: a peer's write into them through its mapping left stale lines in
//          the reader's L2, 8 processes on one MI355X). The next Start's phase 0 keeps every owner
//          from overwriting its outbox before the peers have pulled it.
// The grid never exceeds one workgroup per CU, so every workgroup is resident while any waits.
template <typename T, int OP, int N, int U, int CH>
__global__ __launch_bounds__(EMAC_BLOCK) void ipc_fused_kernel(Work fold, Work pull, emac_codes codes, NodeSync ns,
                                                               unsigned long epoch0, unsigned long epoch1, int nrt) {
  __shared__ int verdict;
  if (threadIdx.x < 64) {
    const bool ok = wave_phase0(ns, epoch0, blockIdx.x == 0);
    if (threadIdx.x == 0) verdict = ok;
  }
  __syncthreads();
  const bool ok = verdict != 0;
  if (ok) run_remote<T, OP, N, U, CH>(fold, codes, nrt);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store of this wave acknowledged
  __syncthreads();
  if (threadIdx.x < 64) {
    unsigned long arrived = 0;
    if (threadIdx.x == 0)
      arrived = __hip_atomic_fetch_add(&ns.self->arrive[ns.slot], 1ul, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    arrived = __shfl(arrived, 0);
    if (arrived == gridDim.x - 1) {  // the last workgroup: every owner chunk of this rank has landed
      // the next launch on this slot is stream-ordered behind this one
      if (threadIdx.x == 0) __hip_atomic_store(&ns.self->arrive[ns.slot], 0ul, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      wave_signal(ns, 1, epoch1, true);
    }
    const bool in_time = wave_wait(ns, 1, epoch1, true);
    const bool gave_up = peer_gave_up(ns);
    wave_report(ns, (in_time ? 0 : EMAC_SYNC_ERR_TIMEOUT) | (gave_up ? EMAC_SYNC_ERR_ABORTED : 0));
    if (threadIdx.x == 0) verdict = ok && in_time && !gave_up;
  }
  __syncthreads();
  if (verdict) run_remote<T, OP, 1, 2, 0>(pull, codes);
}

// ---- instantiation policy (keep in sync with emac_gpu_pick_unroll in fold.hip) ----
// A launch schedule is encoded as U | ISSUE << 4 (sched). SUM, per fold-tree kind CH:
// linear or compile-time chain (gpu.h EMAC_CHAINS), fan-out N (node form):
//        N <= 8 -> (U 2, burst), (U 4, burst), (U 4, s_sleep 2 every 4 loads), (U 1, burst: host
//        buffers), deferred stores (U 2, 4 tiles), (U 4, 2 tiles), (U 2, 8 tiles); N > 8 -> (U 1, burst)
// linear or chain, fan-out 1 (comm form, one-chunk fold): N <= 8 -> U in {1, 2, 4}, burst, and
//        deferred stores (U 2, 4 tiles), (U 4, 4 tiles); N > 8 -> U = 1
// runtime-code tree (composite N, any chain), either fan-out: U = 4 / 2 / 1 for N <= 4 / <= 8 /
//        > 8, burst; U = 2 also with s_sleep 2 every 4 loads (node form)
// peer-mapped (IPC, ISSUE | kRemote): (U 2, burst) up to 8 leaves, (U 1) above; runtime trees U
//        = tree_unroll(N)
// (burst = ISSUE 1: every load of a tile back to back, source-major)
// MIN / MAX: one runtime-leaf-count kernel per element type and fan-out form (N = 0, U = 1).
constexpr int tree_unroll(int n) { return n <= 4 ? 4 : (n <= 8 ? 2 : 1); }
constexpr int sched(int u, int issue) { return u | issue << 4; }

struct Launch {
  const emac_codes *c;
  const emac_bucket *b;
  int nb;
  long ntiles, tpb;
  int all_full;
  const emac_edge *edges;
  int nedges;
  hipStream_t s;
  const unsigned *go;  // peer-mapped launches: the phase-0 verdict word (emac_sync.go[slot])
  int nrt;             // leaves (the runtime-leaf-count kernels)
  bool dry = false;    // resolve the kernel only (emac_gpu_fold_supported): launch nothing
};

template <typename T, int OP, int N, int U, int CH, int D, int ISSUE = 1>
int launch_one(const Launch &L) {
  constexpr int KB = defer_tiles(ISSUE);
  if (L.dry) return 0;
  if constexpr (KB > 1) {  // one workgroup per group of KB tiles
    constexpr bool MAPPED = (ISSUE & kLeafMajor) != 0;  // bucket-mapped groups: the leaf-major ones only
    if (L.tpb == 0 || (L.tpb < 0 && !MAPPED))  // unequal buckets: the per-tile loop
      return launch_one<T, OP, N, U, CH, D, ISSUE & ~(3 << kDeferShift | kLeafMajor | kLmOpenCopy)>(L);
    const long groups = L.tpb < 0 ? L.ntiles : (long)L.nb * ((L.tpb + KB - 1) / KB);
    const unsigned grid = (unsigned)(groups < 8192 ? groups : 8192);
    if (L.tpb < 0) {  // unequal buckets, their first groups in tile0 (layout.c)
      if constexpr (MAPPED) {
        if (L.nb > EMAC_GROUP_MAP_MAX) return EMAC_ERR_ARG;
        if (grid > 0)
          hipLaunchKernelGGL((fold_deferred_map_kernel<T, OP, N, U, CH, D, ISSUE>), dim3(grid), dim3(EMAC_BLOCK), 0, L.s, L.b,
                             L.nb, groups, *L.c);
      }
    } else if (L.all_full && L.tpb % KB == 0)
      hipLaunchKernelGGL((fold_deferred_kernel<T, OP, N, U, CH, D, ISSUE, true>), dim3(grid), dim3(EMAC_BLOCK), 0, L.s, L.b,
                         L.tpb, groups, *L.c);
    else
      hipLaunchKernelGGL((fold_deferred_kernel<T, OP, N, U, CH, D, ISSUE, false>), dim3(grid), dim3(EMAC_BLOCK), 0, L.s, L.b,
                         L.tpb, groups, *L.c);
  } else {
    const long grid = L.ntiles < 8192 ? L.ntiles : 8192;
    if (grid > 0)
      hipLaunchKernelGGL((fold_kernel<T, OP, N, U, CH, D, ISSUE>), dim3((unsigned)grid), dim3(EMAC_BLOCK), 0, L.s, L.b,
                         L.nb, L.ntiles, L.tpb, L.all_full, *L.c, L.go, L.nrt);
  }
  if (L.nedges > 0)
    hipLaunchKernelGGL((fold_edge_kernel<T, OP, N, CH, D, (ISSUE & kRemote) != 0>), dim3((unsigned)L.nedges),
                       dim3(EMAC_BLOCK), 0, L.s, L.b, L.edges, *L.c, L.go, L.nrt);
  return hipGetLastError() == hipSuccess ? 0 : EMAC_ERR_DEVICE;
}

// SUM over N leaves, fold-tree kind CH. FAN: fan-out N (node form); REMOTE: peer-mapped.
template <typename T, int N, bool FAN, bool REMOTE, int CH>
int launch_sum(int unroll, const Launch &L) {
  constexpr int OP = EMAC_SUM;
  constexpr int D = FAN ? N : 1;
  if constexpr (REMOTE) {
    constexpr int UR = CH == 1 ? tree_unroll(N) : (N > 8 ? 1 : 2);
    return unroll == sched(UR, 1 | kRemote) ? launch_one<T, OP, N, UR, CH, D, 1 | kRemote>(L) : EMAC_ERR_UNSUPPORTED;
  } else if constexpr (CH == 1) {
    if (unroll == sched(tree_unroll(N), 1)) return launch_one<T, OP, N, tree_unroll(N), 1, D>(L);
    if constexpr (FAN && tree_unroll(N) == 2) {
      if (unroll == sched(2, 5)) return launch_one<T, OP, N, 2, 1, D, 5>(L);
    }
    return EMAC_ERR_UNSUPPORTED;
  } else if constexpr (N > 8) {
    return unroll == sched(1, 1) ? launch_one<T, OP, N, 1, CH, D>(L) : EMAC_ERR_UNSUPPORTED;
  } else if constexpr (FAN) {
    if (unroll == sched(1, 1)) return launch_one<T, OP, N, 1, CH, D, 1>(L);  // host buffers
    if (unroll == sched(4, 5)) return launch_one<T, OP, N, 4, CH, D, 5>(L);
    if (unroll == sched(4, 1)) return launch_one<T, OP, N, 4, CH, D, 1>(L);
    if (unroll == sched(2, 1)) return launch_one<T, OP, N, 2, CH, D, 1>(L);
    if (unroll == sched(2, 1 | defer(4))) return launch_one<T, OP, N, 2, CH, D, 1 | defer(4)>(L);
    if (unroll == sched(4, 1 | defer(2))) return launch_one<T, OP, N, 4, CH, D, 1 | defer(2)>(L);
    if (unroll == sched(2, 1 | defer(8))) return launch_one<T, OP, N, 2, CH, D, 1 | defer(8)>(L);
    // leaf-major groups: the linear fold and the compile-time chains (CH == 1 took the branch above)
    if (unroll == sched(2, 1 | defer(4) | kLeafMajor)) return launch_one<T, OP, N, 2, CH, D, 1 | defer(4) | kLeafMajor>(L);
    if constexpr (CH > 1) {  // a chain: the opening leaf of each level-0 group copied (kLmOpenCopy)
      if (unroll == sched(2, 1 | defer(4) | kLeafMajor | kLmOpenCopy))
        return launch_one<T, OP, N, 2, CH, D, 1 | defer(4) | kLeafMajor | kLmOpenCopy>(L);
    }
    if constexpr (N == 4 || N == 8) {  // the node fan-outs of 4 and 8 ranks: buffer loads, device-scope stores
      if (unroll == sched(4, 5 | kBufLoad)) return launch_one<T, OP, N, 4, CH, D, 5 | kBufLoad>(L);
      if (unroll == sched(4, 1 | kDevStore | kBufLoad)) return launch_one<T, OP, N, 4, CH, D, 1 | kDevStore | kBufLoad>(L);
    }
    return EMAC_ERR_UNSUPPORTED;
  } else {
    if (unroll == sched(4, 1)) return launch_one<T, OP, N, 4, CH, D>(L);
    if (unroll == sched(2, 1)) return launch_one<T, OP, N, 2, CH, D>(L);
    if (unroll == sched(1, 1)) return launch_one<T, OP, N, 1, CH, D>(L);
    if (unroll == sched(2, 1 | defer(4))) return launch_one<T, OP, N, 2, CH, D, 1 | defer(4)>(L);
    if (unroll == sched(4, 1 | defer(4))) return launch_one<T, OP, N, 4, CH, D, 1 | defer(4)>(L);
    if constexpr (N == 4 || N == 8) {  // one destination of 4 or 8 leaves: (U 4, staggered) with buffer loads
      if (unroll == sched(4, 5 | kBufLoad)) return launch_one<T, OP, N, 4, CH, D, 5 | kBufLoad>(L);
      // (U 4, 2 tiles) of LDS groups: a candidate from 8 MiB per leaf (engine_tune.c; round 6, the
      // local fold forced at 47.6-47.9 us, profiles/r06/localab/, where the LDS groups with buffer
      // loads ran 48.2-48.9 and 8 tiles 48.5-48.8: those are not built)
      if (unroll == sched(4, 1 | defer(2))) return launch_one<T, OP, N, 4, CH, D, 1 | defer(2)>(L);
    }
    return EMAC_ERR_UNSUPPORTED;
  }
}

// the compile-time chains of gpu.h EMAC_CHAINS for N leaves (else the runtime-code kernel)
template <typename T, int N, bool FAN, bool REMOTE>
int launch_sum_ch(int ch, int unroll, const Launch &L) {
  if (ch == 0) return launch_sum<T, N, FAN, REMOTE, 0>(unroll, L);
  if constexpr (can_tree(N)) {
    if (ch == 1) return launch_sum<T, N, FAN, REMOTE, 1>(unroll, L);
  }
  if constexpr (N == 4) {
    if (ch == chain(2, 2)) return launch_sum<T, N, FAN, REMOTE, chain(2, 2)>(unroll, L);
  } else if constexpr (N == 8) {
    if (ch == chain(2, 2, 2)) return launch_sum<T, N, FAN, REMOTE, chain(2, 2, 2)>(unroll, L);
    if (ch == chain(4, 2)) return launch_sum<T, N, FAN, REMOTE, chain(4, 2)>(unroll, L);
    if (ch == chain(2, 4)) return launch_sum<T, N, FAN, REMOTE, chain(2, 4)>(unroll, L);
  } else if constexpr (N == 16) {
    if (ch == chain(2, 2, 2, 2)) return launch_sum<T, N, FAN, REMOTE, chain(2, 2, 2, 2)>(unroll, L);
    if (ch == chain(4, 4)) return launch_sum<T, N, FAN, REMOTE, chain(4, 4)>(unroll, L);
  }
  return EMAC_ERR_UNSUPPORTED;
}

// fan: 0 fan-out 1 (comm form), 1 fan-out N (node form), 2 peer-mapped (IPC form: leaves or the pulled
// result in other GPUs' memory, system-coherent accesses, one destination in this rank's memory)
template <typename T, int N>
int launch_sum_n(int ch, int fan, int unroll, const Launch &L) {
  if constexpr (N == 1) {
    return fan == 2 ? launch_sum<T, 1, false, true, 0>(unroll, L) : launch_sum<T, 1, false, false, 0>(unroll, L);
  } else {
    return fan == 2 ? launch_sum_ch<T, N, false, true>(ch, unroll, L)
                    : fan ? launch_sum_ch<T, N, true, false>(ch, unroll, L) : launch_sum_ch<T, N, false, false>(ch, unroll, L);
  }
}

template <typename T>
int launch_sum_t(int nsrc, int ch, int fan, int unroll, const Launch &L) {
  switch (nsrc) {
#define EMAC_CASE(n) \
  case n: return launch_sum_n<T, n>(ch, fan, unroll, L);
    EMAC_CASE(1) EMAC_CASE(2) EMAC_CASE(3) EMAC_CASE(4) EMAC_CASE(5) EMAC_CASE(6) EMAC_CASE(7) EMAC_CASE(8)
    EMAC_CASE(9) EMAC_CASE(10) EMAC_CASE(11) EMAC_CASE(12) EMAC_CASE(13) EMAC_CASE(14) EMAC_CASE(15) EMAC_CASE(16)
#undef EMAC_CASE
  }
  return EMAC_ERR_UNSUPPORTED;
}

// MIN / MAX: the runtime-leaf-count kernel of the fan-out form (L.nrt leaves)
template <typename T, int OP>
int launch_rt(int fan, int unroll, const Launch &L) {
  if (L.nrt < 1 || L.nrt > kRtMax) return EMAC_ERR_UNSUPPORTED;
  if (fan == 2) return unroll == sched(1, 1 | kRemote) ? launch_one<T, OP, 0, 1, 1, 1, 1 | kRemote>(L) : EMAC_ERR_UNSUPPORTED;
  if (unroll != sched(1, 1)) return EMAC_ERR_UNSUPPORTED;
  return fan ? launch_one<T, OP, 0, 1, 1, 0>(L) : launch_one<T, OP, 0, 1, 1, 1>(L);
}

struct FusedLaunch {
  NodeSync ns;
  unsigned long epoch0, epoch1;
  int grid;
  Work pull;  // every other owner's result into this rank's receive buffer (N = 1, U = 2)
};

template <typename T, int OP, int N, int U, int CH>
int launch_fused_one(const Launch &L, const FusedLaunch &F) {
  const Work fold = {L.b, L.nb, L.ntiles, L.tpb, L.all_full, L.edges, L.nedges};
  hipLaunchKernelGGL((ipc_fused_kernel<T, OP, N, U, CH>), dim3((unsigned)F.grid), dim3(EMAC_BLOCK), 0, L.s, fold, F.pull,
                     *L.c, F.ns, F.epoch0, F.epoch1, L.nrt);
  return hipGetLastError() == hipSuccess ? 0 : EMAC_ERR_DEVICE;
}

// fused peer-mapped launch: the IPC form's schedule of the shape (pick_unroll fan == 2)
template <typename T, int N>
int launch_fused_sum_n(int ch, const Launch &L, const FusedLaunch &F) {
  constexpr int UR = N > 8 ? 1 : 2;
  if (ch == 0) return launch_fused_one<T, EMAC_SUM, N, UR, 0>(L, F);
  if constexpr (can_tree(N)) {
    if (ch == 1) return launch_fused_one<T, EMAC_SUM, N, tree_unroll(N), 1>(L, F);
  }
  if constexpr (N == 4) {
    if (ch == chain(2, 2)) return launch_fused_one<T, EMAC_SUM, N, UR, chain(2, 2)>(L, F);
  } else if constexpr (N == 8) {
    if (ch == chain(2, 2, 2)) return launch_fused_one<T, EMAC_SUM, N, UR, chain(2, 2, 2)>(L, F);
    if (ch == chain(4, 2)) return launch_fused_one<T, EMAC_SUM, N, UR, chain(4, 2)>(L, F);
    if (ch == chain(2, 4)) return launch_fused_one<T, EMAC_SUM, N, UR, chain(2, 4)>(L, F);
  } else if constexpr (N == 16) {
    if (ch == chain(2, 2, 2, 2)) return launch_fused_one<T, EMAC_SUM, N, UR, chain(2, 2, 2, 2)>(L, F);
    if (ch == chain(4, 4)) return launch_fused_one<T, EMAC_SUM, N, UR, chain(4, 4)>(L, F);
  }
  return EMAC_ERR_UNSUPPORTED;
}

template <typename T>
int launch_fused_sum_t(int nsrc, int ch, const Launch &L, const FusedLaunch &F) {
  switch (nsrc) {
#define EMAC_CASE(n) \
  case n: return launch_fused_sum_n<T, n>(ch, L, F);
    EMAC_CASE(2) EMAC_CASE(3) EMAC_CASE(4) EMAC_CASE(5) EMAC_CASE(6) EMAC_CASE(7) EMAC_CASE(8)
    EMAC_CASE(9) EMAC_CASE(10) EMAC_CASE(11) EMAC_CASE(12) EMAC_CASE(13) EMAC_CASE(14) EMAC_CASE(15) EMAC_CASE(16)
#undef EMAC_CASE
  }
  return EMAC_ERR_UNSUPPORTED;
}

template <typename T, int OP>
int launch_fused_rt(const Launch &L, const FusedLaunch &F) {
  if (L.nrt < 2 || L.nrt > kRtMax) return EMAC_ERR_UNSUPPORTED;
  return launch_fused_one<T, OP, 0, 1, 1>(L, F);
}

}  // namespace emac
