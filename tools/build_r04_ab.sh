# Builds the A/B libraries tools/gpu_r04n.sh compares against (CPU side, in-tree under csrc/diag/, travels with the
# tree): the current objects (make first) with one source swapped for an earlier revision, or rebuilt with a flag.
#   bash tools/build_r04_ab.sh        (after: make -C climate-super-resolution_amd/csrc -j8)
set -e
cd "$(dirname "$0")/../climate-super-resolution_amd/csrc"
swap() {  # name, source file, git revision
  mkdir -p diag/$1
  git show $3:climate-super-resolution_amd/csrc/$2 > diag/$1/src.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. -Wall -Wno-unused-function -c diag/$1/src.hip -o diag/$1/src.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o diag/$1/libclimsr_hip.so $(ls *.o | grep -v "^${2%.hip}.o$") diag/$1/src.o
  rm diag/$1/src.o diag/$1/src.hip
  echo "built diag/$1 ($2 @ $3)"
}
swap wrold conv_wr.hip 80a2190    # conv_wr as measured in round 4 (run-time activation, DMA at the tile's start)
swap wrmid conv_wr.hip d8845c0    # templated activation + one-add offsets, DMA still at the tile's start
swap dmaold conv_dma.hip 80a2190  # LDS-DMA conv with the per-element activation
cd ../.. && bash tools/diag_build.sh w64s2old:-DCLIMSR_W64S2_GLDS=0
