// fold_i32_mm.hip -- int MIN / MAX instantiations of the fold kernels (burst schedule only; see
// fold_kernel.hpp). The reference's CPU reduction supports both (ext_mpi_native_exec.c:240-318).
// Compiled twice (Makefile), once per operation (EMAC_MM_OP = 1 for MIN, 2 for MAX), so that the
// two halves build in parallel; the MIN object also carries the dispatch on `op`.
#include "fold_kernel.hpp"

#if EMAC_MM_OP == 1 /* EMAC_MIN (an enum: the preprocessor needs the number) */
extern "C" int emac_fold_launch_i32_max(int nsrc, bool tree, int fan, int unroll, const emac::Launch *L);
extern "C" int emac_fold_fused_launch_i32_max(int nsrc, bool tree, const emac::Launch *L, const emac::FusedLaunch *F);

extern "C" int emac_fold_launch_i32_mm(int op, int nsrc, bool tree, int fan, int unroll, const emac::Launch *L) {
  return op == EMAC_MIN ? emac::launch_t<int, EMAC_MIN>(nsrc, tree, fan, unroll, *L)
                        : emac_fold_launch_i32_max(nsrc, tree, fan, unroll, L);
}

extern "C" int emac_fold_fused_launch_i32_mm(int op, int nsrc, bool tree, const emac::Launch *L,
                                           const emac::FusedLaunch *F) {
  return op == EMAC_MIN ? emac::launch_fused_t<int, EMAC_MIN>(nsrc, tree, *L, *F)
                        : emac_fold_fused_launch_i32_max(nsrc, tree, L, F);
}
#else
extern "C" int emac_fold_launch_i32_max(int nsrc, bool tree, int fan, int unroll, const emac::Launch *L) {
  return emac::launch_t<int, EMAC_MAX>(nsrc, tree, fan, unroll, *L);
}

extern "C" int emac_fold_fused_launch_i32_max(int nsrc, bool tree, const emac::Launch *L, const emac::FusedLaunch *F) {
  return emac::launch_fused_t<int, EMAC_MAX>(nsrc, tree, *L, *F);
}
#endif
