// fold_f32.hip -- float SUM instantiations of the fold kernels (one translation unit per element
// type so that the kernel set compiles in parallel). See fold_kernel.hpp.
#include "fold_kernel.hpp"

extern "C" int emac_fold_launch_f32(int nsrc, int ch, int fan, int unroll, const emac::Launch *L) {
  return emac::launch_sum_t<float>(nsrc, ch, fan, unroll, *L);
}

extern "C" int emac_fold_fused_launch_f32(int nsrc, int ch, const emac::Launch *L, const emac::FusedLaunch *F) {
  return emac::launch_fused_sum_t<float>(nsrc, ch, *L, *F);
}
