// fold_f64_mm.hip -- double MIN / MAX: the runtime-leaf-count kernels of fold_kernel.hpp (one per
// fan-out form). The reference's CPU reduction supports both (ext_mpi_native_exec.c:240-318).
#include "fold_kernel.hpp"

extern "C" int emac_fold_launch_f64_mm(int op, int fan, int unroll, const emac::Launch *L) {
  return op == EMAC_MIN ? emac::launch_rt<double, EMAC_MIN>(fan, unroll, *L) : emac::launch_rt<double, EMAC_MAX>(fan, unroll, *L);
}

extern "C" int emac_fold_fused_launch_f64_mm(int op, const emac::Launch *L, const emac::FusedLaunch *F) {
  return op == EMAC_MIN ? emac::launch_fused_rt<double, EMAC_MIN>(*L, *F) : emac::launch_fused_rt<double, EMAC_MAX>(*L, *F);
}
