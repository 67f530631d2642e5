# A/B libraries for the first round-5 GPU call (CPU side, in-tree under csrc/diag/, travels with the tree): the
# round-4 variants (tools/build_r04_ab.sh) plus diag/main = main's round-4 conv sources (the benched r04 build).
#   make -C climate-super-resolution_amd/csrc -j8 && bash tools/build_r05_ab.sh
set -e
bash "$(dirname "$0")/build_r04_ab.sh"
cd "$(dirname "$0")/../climate-super-resolution_amd/csrc"
mkdir -p diag/main
for f in conv conv_dma conv_wr; do
  git show main:climate-super-resolution_amd/csrc/$f.hip > diag/main/$f.hip
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../../include -I. -Wall -Wno-unused-function -c diag/main/$f.hip -o diag/main/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o diag/main/libclimsr_hip.so elementwise.o disc.o rdb_chain.o rdb_chain_narrow.o data.o rcan.o srcnn.o diag/main/conv.o diag/main/conv_dma.o diag/main/conv_wr.o
rm -f diag/main/*.o diag/main/*.hip
echo "built diag/main"
