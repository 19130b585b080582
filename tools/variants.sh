#!/bin/bash
# Build variants of libhakai_hip.so with extra compile definitions for hakai_kernels.hip, for A/B
# timing in one process tree (HAKAI_LIB=<path> selects the library, hakai/_abi.py):
#   tools/variants.sh name1 "-DFOO" name2 "-DBAR -DBAZ" ...   -> hakai-fem_amd/lib/variants/<name>.so
set -e
cd "$(dirname "$0")/../hakai-fem_amd"
make -s -j8 >/dev/null
mkdir -p lib/variants build/variants
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O3 -fPIC -Wall -Wno-unused-function -munsafe-fp-atomics \
    -ffp-contract=on $defs -c csrc/hakai_kernels.hip -o build/variants/$name.o &
done
wait
for o in build/variants/*.o; do
  name=$(basename $o .o)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib/variants/$name.so $o build/hakai_capi.o build/hakai_comm.o \
    build/hakai_contact.o build/hakai_host.o build/hakai_vtk.o -L/opt/rocm/lib -lrccl -lamdhip64 -pthread
done
ls -la lib/variants
