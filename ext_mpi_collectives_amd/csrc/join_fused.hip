// join_fused.hip -- the peer-mapped node join pipelined by parts in ONE launch per Start
// (engine_join.c, EXT_MPI_AMD_JOIN_PARTS; VERDICT r04 missing 2).
//
// The reference composes a multi-node Allreduce serially: the node's reduce_copyin, the inter-node
// legs, the node's reduce_copyout (src/mpi/ext_mpi_native.c:879-1000). The serial peer-mapped join
// here is three launches and two barriers per Start (engine_join.c node_ipc_init). This kernel cuts
// the message into parts and runs, for part k,
//    CI[k]  the copy-in: the node's R send buffers folded into this node's partial (local HBM),
//    SF[k]  the fold of this node's share of every chunk over the N nodes' partials (peer loads),
//    PL[k]  the pull of every node's share into the R receive buffers (peer loads + local stores),
// in the skewed order CI[0], CI[1], SF[0], CI[2], SF[1], PL[0], ... : every workgroup walks the
// segments in that order, grid-striding over each one's tiles, so while some workgroups still fold
// part k + 1's copy-in (HBM-bound) others fold part k's share and pull part k - 1 (link-bound) --
// what the stream-pipelined join could not do on one MI355X, whose per-part dependent launches and
// cross-stream waits cost 30-110 us each (profiles/r05/join/).
// Dependencies are flags, not launch boundaries:
//  * a workgroup that has finished its tiles of CI[k] drains its stores and counts itself in
//    ctl->ci[k]; the last one signals phase 0 of part k's slot to every node, itself included
//    (ipc_sync.hpp flags: uncached memory, system-scope atomics);
//  * SF[k] waits (one wave per workgroup) for every node's phase 0 of part k; PL[k] for phase 1,
//    which the last workgroup through SF[k] signals the same way;
//  * the copy-in's partial stores are system-coherent write-through (cache policy sc0 sc1), so a
//    peer -- or a workgroup on another XCD of this GPU -- reading the partial after the flag sees
//    it in memory, not in some XCD's L2; the share fold and the pull load with the same policy.
// No workgroup waits for a tile another workgroup has not started: the grid is at most what the
// GPU holds at once (host side), every workgroup folds its copy-in tiles before it waits, and every
// wait is bounded by the communicator's timeout. A part whose phase-0 wait times out is marked
// abandoned in the peers' blocks and its share is not stored; a phase-1 timeout skips the pull's
// stores; both are reported through the slot's error word, as the serial join's barriers do, and
// the next Start synchronises normally (epochs keep counting). The last workgroup out resets the
// control block for the next Start (stream order).
#include <string.h>

#include <type_traits>

#include "fold_kernel.hpp"

namespace emac {

struct JoinSegs {
  Work w[3][EMAC_JOIN_PARTS_MAX];  // [CI, SF, PL][part]
  int slot[EMAC_JOIN_PARTS_MAX];
  unsigned long e0[EMAC_JOIN_PARTS_MAX], e1[EMAC_JOIN_PARTS_MAX];  // this Start's epochs per part
};

// a wave waits for every node's (itself included) flag of `phase` in slot s to reach `epoch`
__device__ __forceinline__ bool join_wait(NodeSync &ns, int phase, unsigned long epoch) {
  return wave_wait(ns, phase, epoch, true);
}

// grid-stride over the tiles and edge items of one segment; N leaves (N = 0: runtime nrt), D
// destinations, ISSUE the load / store policy
template <typename T, int N, int U, int CH, int D, int ISSUE>
__device__ __forceinline__ void join_run(const Work &w, const emac_codes &codes, int nrt, bool store) {
  constexpr long TILE = (long)EMAC_BLOCK * U;
  constexpr long EPV = 16 / sizeof(typename Lane<T>::S);
  constexpr bool REMOTE = (ISSUE & kRemote) != 0;
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
        fold_vectors_rt<T, EMAC_SUM, 1, true, true>(b, t * TILE, 0, codes, nrt, store);
      else
        fold_vectors_rt<T, EMAC_SUM, 1, false, true>(b, t * TILE, b->nvec, codes, nrt, store);
    } else {
      if (w.all_full || (t + 1) * TILE <= b->nvec)
        fold_vectors<T, EMAC_SUM, N, U, CH, D, true, ISSUE>(b, t * TILE, 0, codes, store);
      else
        fold_vectors<T, EMAC_SUM, N, U, CH, D, false, ISSUE>(b, t * TILE, b->nvec, codes, store);
    }
  }
  for (int item = blockIdx.x; item < w.nedges; item += gridDim.x) {
    const emac_edge it = w.edges[item];
    const emac_bucket *b = w.b + it.bucket;
    auto one = [&](long e) {
      if (!store) return;
      if constexpr (N == 0)
        fold_scalar_rt<T, EMAC_SUM, 1, true>(b, e, codes, nrt);
      else
        fold_scalar_element<T, EMAC_SUM, N, CH, D, true>(b, e, codes);
    };
    if (it.mode == 1) {
      for (long e = it.start + threadIdx.x; e < it.start + it.count; e += EMAC_BLOCK) one(e);
    } else {
      const long nsc = b->head + b->tail;
      for (long i = threadIdx.x; i < nsc; i += EMAC_BLOCK) one(i < b->head ? i : b->head + b->nvec * EPV + (i - b->head));
    }
  }
  (void)REMOTE;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's stores acknowledged by memory
}

// this workgroup is through a segment: count it; the last one signals `phase` of the part's slot to
// every node (itself too). Returns nothing; the workgroup's stores were drained before.
__device__ __forceinline__ void join_arrive(unsigned *count, NodeSync &ns, int phase, unsigned long epoch) {
  __shared__ unsigned last;
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x < 64) wave_signal(ns, phase, epoch, true);
}

// wait (one wave) for every node's `phase` of the part; the verdict for the whole workgroup. A
// part some workgroup already found failed is not waited for again (ctl failed word).
__device__ __forceinline__ bool join_gate(NodeSync &ns, int phase, unsigned long epoch, unsigned *failed) {
  __shared__ int verdict;
  if (threadIdx.x < 64) {
    bool ok = __hip_atomic_load(failed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    if (ok) {
      if (!join_wait(ns, phase, epoch)) {
        ok = false;
        wave_report(ns, EMAC_SYNC_ERR_TIMEOUT);
        if (phase == 0) {  // the Start is abandoned on this part: tell every peer (before phase 1)
          const int q = lane_id();
          if (q < ns.nranks && q != ns.me)
            __hip_atomic_store(&ns.peers[q]->aborted[ns.slot][ns.tag & 1], ns.tag, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      } else if (peer_gave_up(ns)) {
        ok = false;
        wave_report(ns, EMAC_SYNC_ERR_ABORTED);
      }
      if (!ok && lane_id() == 0) __hip_atomic_store(failed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x == 0) verdict = ok;
  }
  __syncthreads();
  return verdict != 0;
}

// R copy-in leaves (compile time, fold tree CH), N nodes (runtime, the share's tree in xcodes)
// mode bit 0: the copy-ins; bit 1: the node legs (the signals, waits, share folds and pulls; without
// the copy-ins they read the partials the last ones left -- bench.py times each alone)
template <typename T, int R, int CH>
__global__ __launch_bounds__(EMAC_BLOCK) void join_fused_kernel(JoinSegs segs, int nparts, int mode, emac_codes codes,
                                                                emac_codes xcodes, NodeSync ns0, JoinCtl *ctl) {
  constexpr int CI_ISSUE = 1 | kSysStore;  // local leaves, write-through partial stores
  for (int s = 0; s <= nparts + 1; ++s) {
    if (s < nparts) {  // CI[s]
      NodeSync ns = ns0;
      ns.slot = segs.slot[s];
      ns.tag = segs.e1[s];
      if (mode & 1) join_run<T, R, 2, CH, 1, CI_ISSUE>(segs.w[0][s], codes, 0, true);
      if (mode & 2) join_arrive(&ctl->ci[s], ns, 0, segs.e0[s]);
    }
    if (!(mode & 2)) continue;
    if (s >= 1 && s <= nparts) {  // SF[k]
      const int k = s - 1;
      NodeSync ns = ns0;
      ns.slot = segs.slot[k];
      ns.tag = segs.e1[k];
      const bool ok = join_gate(ns, 0, segs.e0[k], &ctl->failed0[k]);
      join_run<T, 0, 1, 0, 1, 1 | kRemote>(segs.w[1][k], xcodes, ns0.nranks, ok);
      join_arrive(&ctl->sf[k], ns, 1, segs.e1[k]);
    }
    if (s >= 2) {  // PL[k]
      const int k = s - 2;
      NodeSync ns = ns0;
      ns.slot = segs.slot[k];
      ns.tag = segs.e1[k];
      const bool ok = join_gate(ns, 1, segs.e1[k], &ctl->failed1[k]);
      join_run<T, 1, 2, 0, R, 1 | kRemote>(segs.w[2][k], codes, 0, ok);
    }
  }
  // the last workgroup out resets the control block for the next Start (stream-ordered behind)
  __shared__ unsigned last;
  __syncthreads();
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(&ctl->out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x < EMAC_JOIN_PARTS_MAX) {
    ctl->ci[threadIdx.x] = 0;
    ctl->sf[threadIdx.x] = 0;
    ctl->failed0[threadIdx.x] = 0;
    ctl->failed1[threadIdx.x] = 0;
    if (threadIdx.x == 0) ctl->out = 0;
  }
}

template <typename T, int R, int CH>
int join_launch_one(const JoinSegs &segs, int nparts, int mode, const emac_codes &codes, const emac_codes &xcodes,
                    const NodeSync &ns, JoinCtl *ctl, int grid, hipStream_t s) {
  hipLaunchKernelGGL((join_fused_kernel<T, R, CH>), dim3((unsigned)grid), dim3(EMAC_BLOCK), 0, s, segs, nparts, mode,
                     codes, xcodes, ns, ctl);
  return hipGetLastError() == hipSuccess ? 0 : EMAC_ERR_DEVICE;
}

template <typename T, int R>
int join_launch_ch(int ch, const JoinSegs &segs, int nparts, int mode, const emac_codes &codes, const emac_codes &xcodes,
                   const NodeSync &ns, JoinCtl *ctl, int grid, hipStream_t s, bool dry) {
  auto go = [&](auto chc) -> int {
    return dry ? 0 : join_launch_one<T, R, decltype(chc)::value>(segs, nparts, mode, codes, xcodes, ns, ctl, grid, s);
  };
  if (ch == 0) return go(std::integral_constant<int, 0>{});
  if constexpr (R == 4) {
    if (ch == chain(2, 2)) return go(std::integral_constant<int, chain(2, 2)>{});
  } else if constexpr (R == 8) {
    if (ch == chain(2, 2, 2)) return go(std::integral_constant<int, chain(2, 2, 2)>{});
    if (ch == chain(4, 2)) return go(std::integral_constant<int, chain(4, 2)>{});
    if (ch == chain(2, 4)) return go(std::integral_constant<int, chain(2, 4)>{});
  }
  return EMAC_ERR_UNSUPPORTED;
}

template <typename T>
int join_launch_t(int nsrc, int ch, const JoinSegs &segs, int nparts, int mode, const emac_codes &codes, const emac_codes &xcodes,
                  const NodeSync &ns, JoinCtl *ctl, int grid, hipStream_t s, bool dry) {
  switch (nsrc) {
  case 1: return join_launch_ch<T, 1>(ch, segs, nparts, mode, codes, xcodes, ns, ctl, grid, s, dry);
  case 2: return join_launch_ch<T, 2>(ch, segs, nparts, mode, codes, xcodes, ns, ctl, grid, s, dry);
  case 4: return join_launch_ch<T, 4>(ch, segs, nparts, mode, codes, xcodes, ns, ctl, grid, s, dry);
  case 8: return join_launch_ch<T, 8>(ch, segs, nparts, mode, codes, xcodes, ns, ctl, grid, s, dry);
  }
  return EMAC_ERR_UNSUPPORTED;
}

}  // namespace emac

extern "C" int emac_gpu_join_fused(int dtype, int nsrc, const emac_codes *codes, const emac_codes *xcodes, int nparts,
                                   int mode, const emac_join_seg *segs, const int *slots, const unsigned long *e0,
                                   const unsigned long *e1, void *self_sync, void *const *d_peers, int nranks, int me,
                                   int *err, long timeout_ticks, void *ctl, int grid, void *stream) {
  using namespace emac;
  const bool dry = segs == nullptr;
  const int ch = emac_tree_kind(codes, EMAC_SUM);
  if (nparts < 1 || nparts > EMAC_JOIN_PARTS_MAX || codes->nlev > kMaxLevels || xcodes->nlev > kMaxLevels ||
      xcodes->nleaf != nranks || nranks < 1 || nranks > kRtMax)
    return EMAC_ERR_UNSUPPORTED;
  JoinSegs S;
  memset(&S, 0, sizeof(S));
  for (int k = 0; !dry && k < nparts; ++k) {
    for (int st = 0; st < 3; ++st) {
      const emac_join_seg &g = segs[st * EMAC_JOIN_PARTS_MAX + k];
      S.w[st][k] = {g.d_buckets, g.nb, g.ntiles, g.tiles_per_bucket, g.all_full, g.d_edges, g.nedges};
    }
    S.slot[k] = slots[k];
    S.e0[k] = e0[k];
    S.e1[k] = e1[k];
  }
  const NodeSync ns = {static_cast<emac_sync *>(self_sync), reinterpret_cast<emac_sync *const *>(d_peers), 0, nranks, me,
                       err, timeout_ticks, 0};
  hipStream_t s = static_cast<hipStream_t>(stream);
  JoinCtl *c = static_cast<JoinCtl *>(ctl);
  switch (dtype) {
  case EMAC_FLOAT: return join_launch_t<float>(nsrc, ch, S, nparts, mode, *codes, *xcodes, ns, c, grid, s, dry);
  case EMAC_DOUBLE: return join_launch_t<double>(nsrc, ch, S, nparts, mode, *codes, *xcodes, ns, c, grid, s, dry);
  case EMAC_INT: return join_launch_t<int>(nsrc, ch, S, nparts, mode, *codes, *xcodes, ns, c, grid, s, dry);
  case EMAC_LONG: return join_launch_t<long>(nsrc, ch, S, nparts, mode, *codes, *xcodes, ns, c, grid, s, dry);
  }
  return EMAC_ERR_ARG;
}

extern "C" int emac_gpu_join_grid(void) {
  // the workgroups the GPU holds at once of the heaviest instance (8 leaves, float): the grid never
  // exceeds them, so no workgroup waits on tiles of one that cannot start
  int per_cu = 0, dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, emac::join_fused_kernel<float, 8, 0>, EMAC_BLOCK, 0) != hipSuccess ||
      per_cu < 1 || cus < 1)
    return 64;
  return per_cu * cus;
}
