// fold_copy.hip -- the copy-out fan-out of the NODE form over several nodes (and the peer-mapped
// pull that fans each node's share out to the node's receive buffers, emac_gpu_copy_fan_remote)
// (ext_mpi_amd_node_comm_allreduce_init, engine.c): one finished owner chunk stored into the
// node's W other receive buffers, the node allgather of the reference's reduce_copyout stage
// (src/core/reduce_copyin.c:745-838) without a byte over a link: every rank of the node is in
// this GPU's HBM. The streaming fold kernel with one leaf and a compile-time fan-out width
// (fold_kernel.hpp, N = 1, D = W): each leaf vector is read once and stored W times,
// nontemporal. Bits are moved, never combined, so 4- and 8-byte elements of any type go through
// the unsigned integer lanes.
#include "fold_kernel.hpp"

namespace {

template <typename T, int W>
int copy_w(int unroll, const emac::Launch &L) {
  using emac::sched;
  if (unroll == sched(1, 1)) return emac::launch_one<T, EMAC_SUM, 1, 1, 0, W, 1>(L);
  if (unroll == sched(2, 1)) return emac::launch_one<T, EMAC_SUM, 1, 2, 0, W, 1>(L);
  if (unroll == sched(4, 1)) return emac::launch_one<T, EMAC_SUM, 1, 4, 0, W, 1>(L);
  return EMAC_ERR_UNSUPPORTED;
}

// peer-mapped pull with fan-out (engine.c node_ipc_init): the leaf in another GPU's memory, read
// with system-coherent loads (ISSUE kRemote), stored into the node's W receive buffers
template <typename T, int W>
int copy_w_remote(int unroll, const emac::Launch &L) {
  using emac::sched;
  if (unroll == sched(2, 1 | emac::kRemote)) return emac::launch_one<T, EMAC_SUM, 1, 2, 0, W, 1 | emac::kRemote>(L);
  return EMAC_ERR_UNSUPPORTED;
}

template <typename T>
int copy_t_remote(int width, int unroll, const emac::Launch &L) {
  switch (width) {
#define EMAC_CASE(w) \
  case w: return copy_w_remote<T, w>(unroll, L);
    EMAC_CASE(1) EMAC_CASE(2) EMAC_CASE(3) EMAC_CASE(4) EMAC_CASE(5) EMAC_CASE(6) EMAC_CASE(7) EMAC_CASE(8)
    EMAC_CASE(9) EMAC_CASE(10) EMAC_CASE(11) EMAC_CASE(12) EMAC_CASE(13) EMAC_CASE(14) EMAC_CASE(15) EMAC_CASE(16)
#undef EMAC_CASE
  }
  return EMAC_ERR_UNSUPPORTED;
}

template <typename T>
int copy_t(int width, int unroll, const emac::Launch &L) {
  switch (width) {
#define EMAC_CASE(w) \
  case w: return copy_w<T, w>(unroll, L);
    EMAC_CASE(1) EMAC_CASE(2) EMAC_CASE(3) EMAC_CASE(4) EMAC_CASE(5) EMAC_CASE(6) EMAC_CASE(7) EMAC_CASE(8)
    EMAC_CASE(9) EMAC_CASE(10) EMAC_CASE(11) EMAC_CASE(12) EMAC_CASE(13) EMAC_CASE(14) EMAC_CASE(15)
#undef EMAC_CASE
  }
  return EMAC_ERR_UNSUPPORTED;
}

}  // namespace

// width: destinations per bucket (1 .. EMAC_MAX_RANKS - 1); tsize: element bytes (4 or 8)
extern "C" int emac_copy_fan_launch(int tsize, int width, int unroll, const emac::Launch *L) {
  if (tsize == 4) return copy_t<int>(width, unroll, *L);
  if (tsize == 8) return copy_t<long>(width, unroll, *L);
  return EMAC_ERR_ARG;
}

// width 1 .. EMAC_MAX_RANKS, L->go the phase-0 verdict word (a failed barrier skips the stores)
extern "C" int emac_copy_fan_remote_launch(int tsize, int width, int unroll, const emac::Launch *L) {
  if (tsize == 4) return copy_t_remote<int>(width, unroll, *L);
  if (tsize == 8) return copy_t_remote<long>(width, unroll, *L);
  return EMAC_ERR_ARG;
}
