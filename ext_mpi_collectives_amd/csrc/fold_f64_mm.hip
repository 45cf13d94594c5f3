// fold_f64_mm.hip -- double MIN / MAX instantiations of the fold kernels (burst schedule only; see
// fold_kernel.hpp). The reference's CPU reduction supports both (ext_mpi_native_exec.c:240-318).
#include "fold_kernel.hpp"

extern "C" int emac_fold_launch_f64_mm(int op, int nsrc, bool tree, int fan, int unroll, const emac::Launch *L) {
  return op == EMAC_MIN ? emac::launch_t<double, EMAC_MIN>(nsrc, tree, fan, unroll, *L)
                        : emac::launch_t<double, EMAC_MAX>(nsrc, tree, fan, unroll, *L);
}

extern "C" int emac_fold_fused_launch_f64_mm(int op, int nsrc, bool tree, const emac::Launch *L,
                                           const emac::FusedLaunch *F) {
  return op == EMAC_MIN ? emac::launch_fused_t<double, EMAC_MIN>(nsrc, tree, *L, *F)
                        : emac::launch_fused_t<double, EMAC_MAX>(nsrc, tree, *L, *F);
}
