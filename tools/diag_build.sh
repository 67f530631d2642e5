#!/bin/bash
# Diagnostic variants of libclimsr_hip.so (CPU-side build; they travel to the GPU box in-tree) under
# climate-super-resolution_amd/csrc/diag/<name>/libclimsr_hip.so: conv DIAG modes (conv.hip CLIMSR_DIAG_MODE) and
# LDS-DMA conv A/B switches (conv_dma.hip CLIMSR_DMA_*).  Timing experiments only: their results are not valid.
#   bash tools/diag_build.sh conv2:-DCLIMSR_DIAG_MODE=2 dmadirect:-DCLIMSR_DMA_DIRECT=1 ...
set -e
cd "$(dirname "$0")/../climate-super-resolution_amd/csrc"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  out=diag/$name; mkdir -p $out
  for src in $(sed -n 's/^SRCS := //p' Makefile | sed 's/\.hip//g'); do
    extra=""; [ $src = data ] && extra="-ffp-contract=off"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -Wall -Wno-unused-function $extra $flags \
      -c $src.hip -o $out/$src.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $out/libclimsr_hip.so $out/*.o
  rm -f $out/*.o
  echo "built $out/libclimsr_hip.so ($flags)"
done
