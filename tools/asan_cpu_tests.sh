#!/bin/bash
# Host-code sanitizer pass (CPU only): the C engine, planner and layout (plan.c, layout.c,
# engine*.c) rebuilt with -fsanitize=address,undefined and linked with the normal gfx950 kernel
# objects, then the CPU test suite run against that library from a scratch copy of the tree.
# Any "runtime error" / AddressSanitizer report fails the script.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d)
B=$R/ext_mpi_collectives_amd/csrc/build
make -s -C "$R/ext_mpi_collectives_amd/csrc" all
ENG="engine engine_tune engine_node engine_comm engine_ipc engine_join"
for f in plan layout $ENG; do
  gcc -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fPIC -std=gnu11 -D__HIP_PLATFORM_AMD__ \
    -I/opt/rocm/include -I"$R/include" -c "$R/ext_mpi_collectives_amd/csrc/$f.c" -o "$W/$f.o"
done
mkdir -p "$W/tree"
(cd "$R" && git ls-files | tar -cf - -T -) | (cd "$W/tree" && tar -xf -)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fsanitize=address,undefined \
  -o "$W/tree/ext_mpi_collectives_amd/libext_mpi_amd.so" "$W"/plan.o "$W"/layout.o "$W"/engine*.o \
  "$B"/ipc.o "$B"/fold*.o -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib
make -s -C "$R/oracle"
cp "$R/oracle/liboracle.so" "$W/tree/oracle/"
cd "$W/tree"
ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1 \
  LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+:$LD_PRELOAD}" \
  python -m pytest tests -x -q -s -m "not gpu" -p no:cacheprovider --deselect tests/test_mpi_layer.py > "$W/out.txt" 2>&1 || true
tail -1 "$W/out.txt"
if grep -q "runtime error\|ERROR: AddressSanitizer\|failed" "$W/out.txt"; then
  grep -m5 "runtime error\|AddressSanitizer\|failed" "$W/out.txt"
  exit 1
fi
rm -rf "$W"
