#!/bin/bash
# Whole-library variant with extra defines (every source recompiled), built
# out of tree into _lib/libtropical_hip_<name>.so (TNP_LIB selects it):
#   tools/build_full_variant.sh <name> "-DFOO=1 -DBAR=0"
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
name=$1; defs=$2
tmp=$(mktemp -d /tmp/tnp_variant_XXXX)
mkdir -p $tmp/x/csrc $tmp/include
cp $root/tropical-nerf.pytorch_amd/csrc/*.hip $root/tropical-nerf.pytorch_amd/csrc/*.h \
   $root/tropical-nerf.pytorch_amd/csrc/*.cpp $root/tropical-nerf.pytorch_amd/csrc/Makefile $tmp/x/csrc/
cp $root/include/*.h $tmp/include/
make -s -C $tmp/x/csrc -j8 \
  CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-function $defs" \
  OUT=$root/tropical-nerf.pytorch_amd/tropical/_lib/libtropical_hip_$name.so
rm -rf $tmp
echo "built _lib/libtropical_hip_$name.so"
