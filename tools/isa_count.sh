#!/bin/bash
# Instruction counts of the float SUM fold kernels in the gfx950 code object of fold_f32.o:
# per kernel symbol, v_cndmask / v_add_f32 / v_pk_add_f32 / global_load / global_store and the
# total, for the linear fold, the compile-time radix chains and the runtime-code tree.
# Usage: tools/isa_count.sh [object = ext_mpi_collectives_amd/csrc/build/fold_f32.o]
set -e
OBJ=${1:-ext_mpi_collectives_amd/csrc/build/fold_f32.o}
LLVM=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$LLVM/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$OBJ"
$LLVM/clang-offload-bundler --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --output=$T/f32.co --unbundle
$LLVM/llvm-objdump -d --demangle $T/f32.co > $T/f32.s
awk '
/^[0-9a-f]+ <.*>:$/ { name = $0; sub(/^[0-9a-f]+ </, "", name); sub(/>:$/, "", name); next }
name != "" && /v_cndmask/    { cnd[name]++ }
name != "" && /v_add_f32/    { add[name]++ }
name != "" && /v_pk_add_f32/ { pk[name]++ }
name != "" && /global_load/  { ld[name]++ }
name != "" && /global_store/ { st[name]++ }
name != "" && /^[ \t]+[a-z_0-9]+/ { tot[name]++ }
END { for (n in tot) if (n ~ /fold_kernel<float, 0, 8, [24], [0-9]+, 8, [15]>/)
        printf "%6d total %5d v_cndmask %4d v_add_f32 %4d v_pk_add_f32 %4d global_load %4d global_store  %s\n", tot[n], cnd[n], add[n], pk[n], ld[n], st[n], n }
' $T/f32.s | sort -k13
rm -rf $T
