#!/bin/bash
# Faster diagnostic variants: only conv.hip is rebuilt with the variant's flags (all variants in parallel) and linked
# with the in-tree build's other objects (run `make -C climate-super-resolution_amd/csrc` first).  Output:
# climate-super-resolution_amd/csrc/diag/<name>/libclimsr_hip.so.  Timing experiments only.
#   bash tools/diag_build_conv.sh ring0:-DW64_RING=0 w64d1:-DW64_DIAG=1 ...
set -e
cd "$(dirname "$0")/../climate-super-resolution_amd/csrc"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  mkdir -p diag/$name
  ( /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function $flags \
      -c conv.hip -o diag/$name/conv.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o diag/$name/libclimsr_hip.so diag/$name/conv.o \
      elementwise.o disc.o rdb_chain.o data.o rcan.o && rm -f diag/$name/conv.o && echo "built diag/$name ($flags)" ) &
done
wait
