// fold_f64.hip -- double instantiations of the fold kernels (one translation unit per element type so
// that the kernel set compiles in parallel). See fold_kernel.hpp.
#include "fold_kernel.hpp"

extern "C" int emac_fold_launch_f64(int nsrc, bool tree, int fan, int unroll, const emac::Launch *L) {
  return emac::launch_t<double, EMAC_SUM>(nsrc, tree, fan, unroll, *L);
}

extern "C" int emac_fold_fused_launch_f64(int nsrc, bool tree, const emac::Launch *L, const emac::FusedLaunch *F) {
  return emac::launch_fused_t<double, EMAC_SUM>(nsrc, tree, *L, *F);
}
