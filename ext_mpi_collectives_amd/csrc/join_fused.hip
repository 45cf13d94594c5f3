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
// segments in that order, claiming each one's tiles in chunks, so while some workgroups still fold
// part k + 1's copy-in (HBM-bound) others fold part k's share and pull part k - 1 (link-bound) --
// what the stream-pipelined join could not do on one MI355X, whose per-part dependent launches and
// cross-stream waits cost 30-110 us each (profiles/r05/join/).
// Dependencies are flags, not launch boundaries:
//  * a workgroup that has finished its items of CI[k] drains its stores and counts them in
//    ctl->done; the one that completes the count signals phase 0 of part k's slot to every node,
//    itself included (ipc_sync.hpp flags: uncached memory, system-scope atomics);
//  * SF[k] waits (one wave per workgroup) for every node's phase 0 of part k; PL[k] for phase 1,
//    which the last workgroup through SF[k] signals the same way;
//  * the copy-in's partial stores are system-coherent write-through (cache policy sc0 sc1), so a
//    peer -- or a workgroup on another XCD of this GPU -- reading the partial after the flag sees
//    it in memory, not in some XCD's L2; the share fold and the pull load with the same policy.
// No workgroup waits for an item a workgroup that has not started holds: items are claimed from a
// counter by running workgroups only (join_seg), and every wait is bounded by the communicator's
// timeout. A part whose phase-0 wait times out is marked
// abandoned in the peers' blocks and its share is not stored; a phase-1 timeout skips the pull's
// stores; both are reported through the slot's error word, as the serial join's barriers do, and
// the next Start synchronises normally (epochs keep counting). The last workgroup out resets the
// control block for the next Start (stream order).
// One relaxation of the serial join's rule (a rank that times out in phase 0 folds nothing): here the
// verdict is per workgroup. A workgroup that passed the phase-0 gate before another one timed out
// and published the abandon marks still folds and stores its share items. Nothing is corrupted --
// those stores go only to this node's own outbox, and the Start is reported failed on every node
// through the marks and the slot's error word -- but part of a failed Start's share may be stored.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <type_traits>

#include "fold_kernel.hpp"

namespace emac {

// 1024-lane workgroups, one per CU: 16 waves per CU without more workgroups contending for the
// segments' counters (each one claims and counts on them; 4x the workgroups of 256 lanes cost 40-170
// us more per Start at 512-2048 workgroups, profiles/r05/join/). A tile is JB * U vectors: the
// layouts are made with U * JB / EMAC_BLOCK (engine_join.c).
constexpr int JB = 1024;

struct JoinSegs {
  Work w[3][EMAC_JOIN_PARTS_MAX];  // [CI, SF, PL][part]
  int slot[EMAC_JOIN_PARTS_MAX];
  unsigned long e0[EMAC_JOIN_PARTS_MAX], e1[EMAC_JOIN_PARTS_MAX];  // this Start's epochs per part
  unsigned long *trace;  // diagnostics (EXT_MPI_AMD_JOIN_TRACE): kTraceSlots per workgroup, or null
};

// Diagnostics: with EXT_MPI_AMD_JOIN_TRACE=<path> every workgroup's thread 0 records the wall clock
// (100 MHz) when it starts, leaves each segment or passes a gate, and ends, as
// (clock << 16) | (items << 8) | tag, tag = stage << 4 | part (stage 0 CI, 1 SF gate, 2 SF, 3 PL gate,
// 4 PL; 14 start, 15 end); the host appends each launch's records to <path>.<pid> before the next
// launch (which then waits for it: a diagnostic of one launch's timeline, not of Start-to-Start overlap)
constexpr int kTraceSlots = 32;

// a wave waits for every node's (itself included) flag of `phase` in slot s to reach `epoch`
__device__ __forceinline__ bool join_wait(NodeSync &ns, int phase, unsigned long epoch) {
  return wave_wait(ns, phase, epoch, true);
}

// one item of a segment: tile `i` (i < ntiles) or edge item i - ntiles; N leaves (N = 0: runtime
// nrt), D destinations, ISSUE the load / store policy
template <typename T, int N, int U, int CH, int D, int ISSUE>
__device__ __forceinline__ void join_item(const Work &w, long i, const emac_codes &codes, int nrt, bool store) {
  constexpr long TILE = (long)JB * U;
  constexpr long EPV = 16 / sizeof(typename Lane<T>::S);
  if (i < w.ntiles) {
    const long tile = i;
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
        fold_vectors<T, EMAC_SUM, N, U, CH, D, true, ISSUE, JB>(b, t * TILE, 0, codes, store);
      else
        fold_vectors<T, EMAC_SUM, N, U, CH, D, false, ISSUE, JB>(b, t * TILE, b->nvec, codes, store);
    }
    return;
  }
  if (!store) return;
  const emac_edge it = w.edges[i - w.ntiles];
  const emac_bucket *b = w.b + it.bucket;
  auto one = [&](long e) {
    if constexpr (N == 0)
      fold_scalar_rt<T, EMAC_SUM, 1, true>(b, e, codes, nrt);
    else
      fold_scalar_element<T, EMAC_SUM, N, CH, D, true>(b, e, codes);
  };
  if (it.mode == 1) {
    for (long e = it.start + threadIdx.x; e < it.start + it.count; e += JB) one(e);
  } else {
    const long nsc = b->head + b->tail;
    for (long j = threadIdx.x; j < nsc; j += JB) one(j < b->head ? j : b->head + b->nvec * EPV + (j - b->head));
  }
}

// The items of one segment, claimed in chunks from the segment's ticket counter (the next chunk's
// ticket fetched while the current one is folded, where that cannot starve another workgroup); then this workgroup's items are counted in
// `done`, and whoever completes the count -- for a segment of no item, the first through -- signals
// `phase` of the part's slot to every node, itself too (phase < 0: nothing to signal). Claiming
// rather than a static grid stride: a workgroup the GPU has not started yet holds no item a
// waiting one needs, so the grid need not be resident all at once.
template <typename T, int N, int U, int CH, int D, int ISSUE>
__device__ __forceinline__ unsigned join_seg(const Work &w, unsigned *tk, unsigned *done, unsigned *sig, const emac_codes &codes,
                                             int nrt, bool store, NodeSync &ns, int phase, unsigned long epoch) {
  __shared__ unsigned claim[2];
  __shared__ unsigned last;
  const unsigned n = (unsigned)(w.ntiles + w.nedges);
  unsigned c = n / (gridDim.x * 4u);  // a few chunks per workgroup: few claims, balanced ends
  c = c < 1u ? 1u : c > 32u ? 32u : c;
  unsigned mine = 0;
  __syncthreads();
  if (threadIdx.x == 0) claim[0] = n ? __hip_atomic_fetch_add(tk, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
  __syncthreads();
  unsigned at = claim[0];
  while (at < n) {
    unsigned next = 0;
    // the next chunk is fetched while this one is folded only while more than a grid's worth of
    // chunks follows it: fetched early in a segment of about one chunk per workgroup, it let the
    // first workgroups take two chunks each and left others none -- two tiles in series on the
    // critical path (join_trace_summary.py: items per workgroup 0-2 in a segment of grid items)
    const bool ahead = (unsigned long)at + (unsigned long)c * gridDim.x < n;
    if (threadIdx.x == 0 && ahead) next = __hip_atomic_fetch_add(tk, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned end = at + c < n ? at + c : n;
    for (unsigned i = at; i < end; ++i) join_item<T, N, U, CH, D, ISSUE>(w, (long)i, codes, nrt, store);
    if (threadIdx.x == 0 && !ahead) next = __hip_atomic_fetch_add(tk, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    mine += end - at;
    __syncthreads();
    if (threadIdx.x == 0) claim[1] = next;
    __syncthreads();
    at = claim[1];
  }
  // a segment whose completion is signalled: this workgroup's stores acknowledged by memory before
  // it counts them. A segment that signals nothing (the pulls; the copy-ins timed alone) is not
  // counted at all: its stores complete with the launch, and the workgroup goes on at once
  // instead of waiting for a counter's round trip
  if (phase < 0) return mine;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // (one counter per segment for the whole grid: its atomics serialise -- a segment of no item, where
  // every workgroup once added 0 and exchanged the flag, took 5-8 us (join_trace_summary.py) -- so
  // a workgroup of no item does not count, and with no item at all the flag is read before it is
  // taken: only the first workgroups through try the exchange)
  if (threadIdx.x == 0) {
    if (n == 0) {
      last = __hip_atomic_load(sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
             __hip_atomic_exchange(sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    } else if (mine) {
      const unsigned before = __hip_atomic_fetch_add(done, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = before + mine == n && __hip_atomic_exchange(sig, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    } else {
      last = false;  // the workgroup that completes the count holds items
    }
  }
  __syncthreads();
  if (last && threadIdx.x < 64) wave_signal(ns, phase, epoch, true);
  return mine;
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
// The copy-in's tiles are JB * 2 vectors of one bucket (engine_join.c lays them out so). Wider and
// narrower ones were measured on configs[1]'s node, the copy-ins alone (bench.py --shape joinci,
// profiles/r06/joinci/): 2 parts, 39.3 us at 2 vectors per lane, 40.6 at 1 (one claim per workgroup
// and part), 41.8 at 3, 46.9 at 4 -- more loads in flight per wave made it slower.
template <typename T, int R, int CH, bool SYS>
__global__ __launch_bounds__(JB) void join_fused_kernel(JoinSegs segs, int nparts, int mode, emac_codes codes,
                                                                emac_codes xcodes, NodeSync ns0, JoinCtl *ctl) {
  // local leaves, read with nontemporal buffer loads (kBufLoad: the copy-in alone 35.5-36.4 us
  // against 36.8-36.9 with global loads, Starts with 2 / 4 nodes on one GPU equal or 1-2 % faster;
  // staggered issue and vector-major order were not better, profiles/r06/ciload/); the partial
  // written through to memory, at system scope when a peer runs on another GPU, else at device
  // scope (kDevStore: sc1 nt) -- enough for this GPU's other XCDs and processes
  constexpr int CI_ISSUE = 1 | kBufLoad | (SYS ? kSysStore : kDevStore);
  unsigned long *const tr = segs.trace ? segs.trace + (size_t)blockIdx.x * kTraceSlots : nullptr;
  int ev = 0;
  auto mark = [&](unsigned tag, unsigned items) {  // (wave-uniform branch on tr)
    if (tr && threadIdx.x == 0 && ev < kTraceSlots)
      tr[ev] = (unsigned long)wall_clock64() << 16 | (unsigned long)(items > 255u ? 255u : items) << 8 | tag;
    ++ev;
  };
  mark(14u << 4, 0);
  for (int s = 0; s <= nparts + 1; ++s) {
    if (s < nparts) {  // CI[s]: signals phase 0 of part s when its last item is in (with the node legs)
      NodeSync ns = ns0;
      ns.slot = segs.slot[s];
      ns.tag = segs.e1[s];
      const Work empty = {segs.w[0][s].b, 0, 0, 0, 1, nullptr, 0};
      const unsigned it = join_seg<T, R, 2, CH, 1, CI_ISSUE>((mode & 1) ? segs.w[0][s] : empty, &ctl->tk[0][s], &ctl->done[0][s],
                                         &ctl->sig[0][s], codes, 0, true, ns, (mode & 2) ? 0 : -1, segs.e0[s]);
      mark(0u << 4 | s, it);
    }
    if (!(mode & 2)) continue;
    if (s >= 1 && s <= nparts) {  // SF[k], after every node's phase 0 of part k; signals phase 1
      const int k = s - 1;
      NodeSync ns = ns0;
      ns.slot = segs.slot[k];
      ns.tag = segs.e1[k];
      const bool ok = join_gate(ns, 0, segs.e0[k], &ctl->failed0[k]);
      mark(1u << 4 | k, 0);
      const unsigned it = join_seg<T, 0, 1, 0, 1, 1 | kRemote | kNoDrain>(segs.w[1][k], &ctl->tk[1][k], &ctl->done[1][k],
                                                                        &ctl->sig[1][k], xcodes, ns0.nranks, ok, ns, 1, segs.e1[k]);
      mark(2u << 4 | k, it);
    }
    if (s >= 2) {  // PL[k], after every node's phase 1 of part k
      const int k = s - 2;
      NodeSync ns = ns0;
      ns.slot = segs.slot[k];
      ns.tag = segs.e1[k];
      const bool ok = join_gate(ns, 1, segs.e1[k], &ctl->failed1[k]);
      mark(3u << 4 | k, 0);
      const unsigned it = join_seg<T, 1, 2, 0, R, 1 | kRemote | kNoDrain>(segs.w[2][k], &ctl->tk[2][k], &ctl->done[2][k],
                                                                        &ctl->sig[2][k], codes, 0, ok, ns, -1, 0);
      mark(4u << 4 | k, it);
    }
  }
  mark(15u << 4, 0);
  // the last workgroup out resets the control block for the next Start (stream-ordered behind)
  __shared__ unsigned last;
  __syncthreads();
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(&ctl->out, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (last) {
    unsigned *cw = reinterpret_cast<unsigned *>(ctl);
    for (unsigned i = threadIdx.x; i < sizeof(JoinCtl) / sizeof(unsigned); i += JB) cw[i] = 0;
  }
}

template <typename T, int R, int CH>
int join_launch_one(const JoinSegs &segs, int nparts, int mode, const emac_codes &codes, const emac_codes &xcodes,
                    const NodeSync &ns, JoinCtl *ctl, int grid, hipStream_t s) {
  if (mode & 4)  // every node on this GPU: device-scope write-through suffices
    hipLaunchKernelGGL((join_fused_kernel<T, R, CH, false>), dim3((unsigned)grid), dim3(JB), 0, s, segs, nparts,
                       mode, codes, xcodes, ns, ctl);
  else
    hipLaunchKernelGGL((join_fused_kernel<T, R, CH, true>), dim3((unsigned)grid), dim3(JB), 0, s, segs, nparts,
                       mode, codes, xcodes, ns, ctl);
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

namespace {
// EXT_MPI_AMD_JOIN_TRACE (see kTraceSlots): the previous launch's records appended to the file, this
// launch's buffer cleared; null when off
unsigned long *join_trace_next(int grid, int mode, hipStream_t s) {
  using namespace emac;
  static int on = -1, prev_grid = 0, prev_mode = 0;
  static long launches = 0;
  static unsigned long *d = nullptr, *h = nullptr;
  static FILE *f = nullptr;
  constexpr int kMaxGrid = 4096;
  if (on < 0) {
    const char *e = getenv("EXT_MPI_AMD_JOIN_TRACE");
    on = e && *e;
    if (on) {
      char path[512];
      snprintf(path, sizeof(path), "%s.%d", e, (int)getpid());
      f = fopen(path, "a");
      h = static_cast<unsigned long *>(malloc(sizeof(unsigned long) * kMaxGrid * kTraceSlots));
      if (!f || !h || hipMalloc(reinterpret_cast<void **>(&d), sizeof(unsigned long) * kMaxGrid * kTraceSlots) != hipSuccess)
        on = 0;
    }
  }
  if (!on || grid > kMaxGrid) return nullptr;
  if (launches > 0 && hipStreamSynchronize(s) == hipSuccess &&
      hipMemcpy(h, d, sizeof(unsigned long) * prev_grid * kTraceSlots, hipMemcpyDeviceToHost) == hipSuccess) {
    fprintf(f, "launch %ld mode %d grid %d\n", launches - 1, prev_mode, prev_grid);
    for (int g = 0; g < prev_grid; ++g) {
      fprintf(f, "%d", g);
      for (int k = 0; k < kTraceSlots && h[(size_t)g * kTraceSlots + k]; ++k) fprintf(f, " %lu", h[(size_t)g * kTraceSlots + k]);
      fprintf(f, "\n");
    }
    fflush(f);
  }
  (void)hipMemsetAsync(d, 0, sizeof(unsigned long) * grid * kTraceSlots, s);
  prev_grid = grid;
  prev_mode = mode;
  ++launches;
  return d;
}
}  // namespace

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
  if (!dry) S.trace = join_trace_next(grid, mode, s);
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
  // one workgroup per CU (items are claimed, so the grid need not match the work): every segment
  // costs each workgroup a claim and a count on the segment's counters, and a wider grid only adds
  // contention on them (EXT_MPI_AMD_JOIN_GRID overrides, for A/B runs)
  int dev = 0, cus = 0;
  const char *e = getenv("EXT_MPI_AMD_JOIN_GRID");
  if (e && atoi(e) > 0) return atoi(e);
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus < 1)
    return 256;
  return cus;
}
